// hq_fused.hip — software-pipelined fused map + streaming index + embed + uint8 quantize for the
// common grid sides (16, 32, 64) and index lengths L <= 64.  Same contract and bit-exact results
// as k_fused (hq_quant.hip); SURVEY.md §8a rows M5, P1, I1, I3, Q1.
//
// Reference sequence: core/pipeline.py:97-146 (pad -> map_to_2d -> streaming index -> embed ->
// _normalize_for_compression), index tree core/streaming_index_builder.py:45-243.
//
// Structure (one wave64 per embedding, persistent grid, HBM-bound):
//   * lane j owns float4 groups j + 64t (t < ND = data groups per lane); loads are coalesced 1 KiB
//     wave instructions and the NEXT embedding's groups are loaded before the current one is
//     processed (explicit A/B register ping-pong), so HBM latency overlaps the arithmetic;
//   * tree level 1 is a float4 group (registers), level 2 is a quad reduction with DPP quad_perm
//     broadcasts (same left-to-right f64 order), levels >= 3 are tiny LDS reductions;
//   * every index slot i < L is owned by lane i, which knows its (level, position) from a host
//     plan: level-0 / level-1 slots load their own element / group with the prefetch, deeper slots
//     read the LDS tree — no global re-reads and no second min/max reduction (all index values lie
//     inside [min, max] of the padded data, core/index_generator.py:247 casts them to f32; only the
//     zero fill of unused index-row slots can extend the range, decided on the host);
//   * 2x2 blocks of the image are float4 groups, so each lane scatters two u16 pairs into a
//     row-major LDS frame that is streamed out with 16-byte stores.
#include "hq_common.h"

#include <stdlib.h>

namespace hq {

struct FastPlan {
  int8_t lev[64];   // slot level (-1: zero fill)
  int32_t pos[64];  // position inside the level
  int zero_row;     // index row holds zero-fill slots among its first n entries
};

template <int CTRL>
__device__ __forceinline__ double quad_bcast(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double quad_bcast_xor1(double v) {  // value of lane ^ 1 (quad_perm 1,0,3,2)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// index row store with 16-byte lanes: even lanes write (slot 2k, slot 2k+1) — 8-byte stores leave
// L2 at a much lower byte rate (MI355X_MICROARCH.md, store flavours); L even and 16-B aligned rows
template <bool NT = false>
__device__ __forceinline__ void store_index(double* __restrict__ row, double val, int lane, int L) {
  const double nb = quad_bcast_xor1(val);
  if ((L & 1) == 0 && (reinterpret_cast<uintptr_t>(row) & 15) == 0) {
    if ((lane & 1) == 0 && lane < L) {
      if constexpr (NT) {
        typedef double d2v __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(d2v{val, nb}, reinterpret_cast<d2v*>(row + lane));
      } else {
        *reinterpret_cast<double2*>(row + lane) = make_double2(val, nb);
      }
    }
  } else if (lane < L) {
    row[lane] = val;
  }
}
__device__ __forceinline__ uint32_t qz(float x, float mn, float rng) {
  float t = (x - mn) / rng;  // IEEE f32 division (no fast-math), then * 255 and truncate
  t = t * 255.0f;
  return (uint32_t)t;
}
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float* p) {  // read-once stream: non-temporal
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

template <int NS>
struct FastGeo {
  static constexpr int G = NS * NS / 4;
  static constexpr int NT = G / 64;
  static constexpr int FB = (NS + 1) * NS;
  static constexpr int levels() {
    int k = 0, s = NS * NS;
    while (k < kStreamMaxLevels && s > 0) { ++k; s >>= 2; }
    return k;
  }
  // LDS tree holds levels >= 2; level l (>= 2) has G >> (2(l-1)) values
  static constexpr int off(int l) {
    int t = 0, s = G >> 2;
    for (int k = 2; k < l; ++k) { t += s; s >>= 2; }
    return t;
  }
  static constexpr int tree_len() { return off(levels()); }
  static constexpr int frame_off() { return ((tree_len() * 8 + G * 4) + 15) & ~15; }
  static constexpr size_t lds_bytes() { return (size_t)frame_off() + ((FB + 15) & ~15); }
};

template <int NS, int ND>
struct Buf {
  float4 g[ND];
  float4 slot;
};

template <int NS, int ND, int V>
__device__ __forceinline__ void load_emb(const float* __restrict__ src, int d, int lane, int slev, int spos,
                                         Buf<NS, ND>& b) {
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    const int j = lane + 64 * t;
    if (4 * j + 3 < d) {
      if constexpr ((V & 1) != 0) b.g[t] = ld_stream(src + 4 * j);
      else b.g[t] = *reinterpret_cast<const float4*>(src + 4 * j);
    } else {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (4 * j + 0 < d) x.x = src[4 * j + 0];
      if (4 * j + 1 < d) x.y = src[4 * j + 1];
      if (4 * j + 2 < d) x.z = src[4 * j + 2];
      b.g[t] = x;
    }
  }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (slev == 0) {
    if (spos < d) s.x = src[spos];
  } else if (slev == 1) {
    const int p = 4 * spos;
    if (p + 3 < d) {
      s = *reinterpret_cast<const float4*>(src + p);
    } else {
      if (p + 0 < d) s.x = src[p + 0];
      if (p + 1 < d) s.y = src[p + 1];
      if (p + 2 < d) s.z = src[p + 2];
    }
  }
  b.slot = s;
}

template <int NS, int ND, int V>
__device__ __forceinline__ void process_emb(int64_t e, const Buf<NS, ND>& b, int d, int L, int lane, int slev,
                                            int spos, bool pad0, double* tree, const uint32_t (&lut_r)[ND], uint8_t* frame,
                                            uint8_t* __restrict__ frame_out, double* __restrict__ idx_out,
                                            float* __restrict__ mm_out, bool live = true) {
  using Geo = FastGeo<NS>;
  constexpr int NLEV = Geo::levels();
  // memory-only probes (HQ_FUSED_V = 8 / 12: the kernel's full traffic with no arithmetic; + 16: no frame
  // stores, + 32: no index / min-max stores) bound what the arithmetic costs: V 8 runs within ~4 % of V 4
  if constexpr ((V & 8) != 0) {
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < ND; ++t) acc += (b.g[t].x + b.g[t].y) + (b.g[t].z + b.g[t].w);
    if constexpr ((V & 32) == 0) {
      store_index(idx_out + e * (int64_t)L, (double)acc, lane, L);
      if (mm_out && lane == 0) mm_out[2 * e] = acc;
    } else {
      if (acc == 1234.5f) idx_out[0] = 0.0;  // keep the loads
    }
    if constexpr ((V & 16) == 0) {
      uint8_t* dst = frame_out + e * (int64_t)Geo::FB;
#pragma unroll
      for (int c = lane; c < Geo::FB / 16; c += 64)
        reinterpret_cast<uint4*>(dst)[c] = reinterpret_cast<const uint4*>(frame)[c];
    }
    return;
  }
  // ---- min / max over the real elements --------------------------------------------------------
  float lmin = __builtin_huge_valf(), lmax = -__builtin_huge_valf();
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    const int j = lane + 64 * t;
    const float4 x = b.g[t];
    if (4 * j + 3 < d) {
      lmin = fminf(lmin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
      lmax = fmaxf(lmax, fmaxf(fmaxf(x.x, x.y), fmaxf(x.z, x.w)));
    } else {
      if (4 * j + 0 < d) { lmin = fminf(lmin, x.x); lmax = fmaxf(lmax, x.x); }
      if (4 * j + 1 < d) { lmin = fminf(lmin, x.y); lmax = fmaxf(lmax, x.y); }
      if (4 * j + 2 < d) { lmin = fminf(lmin, x.z); lmax = fmaxf(lmax, x.z); }
    }
  }
  float mn = wmin64(lmin), mx = wmax64(lmax);
  if (pad0) { mn = fminf(mn, 0.f); mx = fmaxf(mx, 0.f); }

  // ---- tree: level 1 in registers, level 2 by quad DPP, deeper levels in LDS ---------------------
  if (NLEV > 2) {
#pragma unroll
    for (int t = 0; t < ND; ++t) {
      const float4 x = b.g[t];
      const double l1 = ((((double)x.x + (double)x.y) + (double)x.z) + (double)x.w) * 0.25;
      const double a0 = quad_bcast<0x00>(l1), a1 = quad_bcast<0x55>(l1);
      const double a2 = quad_bcast<0xAA>(l1), a3 = quad_bcast<0xFF>(l1);
      const double l2 = (((a0 + a1) + a2) + a3) * 0.25;
      if ((lane & 3) == 0) tree[Geo::off(2) + (lane >> 2) + 16 * t] = l2;
    }
    __syncthreads();
#pragma unroll
    for (int l = 3; l < NLEV; ++l) {
      const int S = Geo::G >> (2 * (l - 1));
      const double* a = tree + Geo::off(l - 1);
      double* o = tree + Geo::off(l);
      for (int k = lane; k < S; k += 64) o[k] = (((a[4 * k] + a[4 * k + 1]) + a[4 * k + 2]) + a[4 * k + 3]) * 0.25;
      __syncthreads();
    }
  }

  // ---- this lane's index slot ------------------------------------------------------------------
  double val = 0.0;
  if (slev == 0) {
    val = (double)b.slot.x;
  } else if (slev == 1) {
    val = ((((double)b.slot.x + (double)b.slot.y) + (double)b.slot.z) + (double)b.slot.w) * 0.25;
  } else if (slev >= 2) {
    val = tree[Geo::off(slev) + spos];
  }
  if (live) store_index<(V & 2048) != 0>(idx_out + e * (int64_t)L, val, lane, L);
  const float rv = (float)val;
  if constexpr ((V & 512) != 0) __syncthreads();  // frame overlays the tree: every slot read first

  // ---- quantize into the LDS frame, stream out --------------------------------------------------
  const bool flat = mx == mn;
  const float rng = mx - mn;
  const uint32_t q0 = flat ? 128u : qz(0.f, mn, rng);
  const int groups_data = (d + 3) >> 2;
  if (d < NS * NS || flat) {
    const uint32_t w = q0 * 0x01010101u;
    const uint4 w4 = make_uint4(w, w, w, w);
#pragma unroll
    for (int c = lane; c < NS * NS / 16; c += 64) reinterpret_cast<uint4*>(frame)[c] = w4;
  }
  if (!flat) {
    const float rcp = 1.0f / rng;
    const float c255 = rcp * 255.0f;
    (void)c255;
#pragma unroll
    for (int t = 0; t < ND; ++t) {
      const int j = lane + 64 * t;
      if (j < groups_data) {
        const float4 x = b.g[t];
        const uint32_t ent = lut_r[t];
        const uint32_t code = ent >> 16;
        uint32_t w;
        if constexpr ((V & 2) != 0) {
          // packed f32 pairs: y = (x - mn) * fl(fl(1/rng) * 255) (qfast's < 7.7e-5 bound), floor(y)
          // placed straight into its 2x2-block byte by v_cvt_pk_u8_f32; the exact division only at an
          // element position where some lane's y lies within 1e-4 of an integer
          typedef float f2v __attribute__((ext_vector_type(2)));
          const f2v mn2 = {mn, mn}, c2 = {c255, c255}, h2 = {0.5f, 0.5f};
          const f2v ya = (f2v{x.x, x.y} - mn2) * c2, yb = (f2v{x.z, x.w} - mn2) * c2;
          f2v fa = {floorf(ya.x), floorf(ya.y)}, fb = {floorf(yb.x), floorf(yb.y)};
          const f2v ta = (ya - fa) - h2, tb = (yb - fb) - h2;
          const float q0f = (float)q0;
          if (4 * j + 3 >= d) {  // the group that straddles d: padding elements quantize 0.0
            if (4 * j + 1 >= d) fa.y = q0f;
            if (4 * j + 2 >= d) fb.x = q0f;
            fb.y = q0f;
          }
          const float xs[4] = {x.x, x.y, x.z, x.w};
          const bool sl[4] = {fabsf(ta.x) > 0.4999f, fabsf(ta.y) > 0.4999f && 4 * j + 1 < d,
                              fabsf(tb.x) > 0.4999f && 4 * j + 2 < d, fabsf(tb.y) > 0.4999f && 4 * j + 3 < d};
          const uint32_t p0 = code & 3u, p1 = (code >> 2) & 3u, p2 = (code >> 4) & 3u, p3 = (code >> 6) & 3u;
          w = __builtin_amdgcn_cvt_pk_u8_f32(fa.x, p0, 0u);
          w = __builtin_amdgcn_cvt_pk_u8_f32(fa.y, p1, w);
          w = __builtin_amdgcn_cvt_pk_u8_f32(fb.x, p2, w);
          w = __builtin_amdgcn_cvt_pk_u8_f32(fb.y, p3, w);
          const uint32_t ps[4] = {p0, p1, p2, p3};
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (__builtin_amdgcn_ballot_w64(sl[m]))
              if (sl[m]) w = (w & ~(0xFFu << (8 * ps[m]))) | (qz(xs[m], mn, rng) << (8 * ps[m]));
        } else {
          const uint32_t e0 = qz(x.x, mn, rng);
          const uint32_t e1 = (4 * j + 1 < d) ? qz(x.y, mn, rng) : q0;
          const uint32_t e2 = (4 * j + 2 < d) ? qz(x.z, mn, rng) : q0;
          const uint32_t e3 = (4 * j + 3 < d) ? qz(x.w, mn, rng) : q0;
          w = (e0 << (8 * (code & 3))) | (e1 << (8 * ((code >> 2) & 3))) | (e2 << (8 * ((code >> 4) & 3))) |
              (e3 << (8 * ((code >> 6) & 3)));
        }
        const uint32_t off = ent & 0xFFFFu;
        *reinterpret_cast<uint16_t*>(frame + off) = (uint16_t)(w & 0xFFFFu);
        *reinterpret_cast<uint16_t*>(frame + off + NS) = (uint16_t)(w >> 16);
      }
    }
  }
  if (lane < NS) frame[NS * NS + lane] = flat ? (uint8_t)128 : (uint8_t)qz(rv, mn, rng);
  __syncthreads();
  uint8_t* dst = frame_out + e * (int64_t)Geo::FB;
  if (live) {
#pragma unroll
    for (int c = lane; c < Geo::FB / 16; c += 64) {
      if constexpr ((V & 1024) != 0) {  // non-temporal frame stores (A/B)
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(reinterpret_cast<const u4v*>(frame)[c], reinterpret_cast<u4v*>(dst) + c);
      } else {
        reinterpret_cast<uint4*>(dst)[c] = reinterpret_cast<const uint4*>(frame)[c];
      }
    }
    if (mm_out && lane == 0) *reinterpret_cast<float2*>(mm_out + 2 * e) = make_float2(mn, mx);
  }
  if constexpr ((V & 64) == 0) __syncthreads();  // persistent: the frame is reused by the next embedding
}

template <int NS, int ND, int V>
__global__ __launch_bounds__(64) void k_fused_fast(const float* __restrict__ in, int64_t N, int64_t stride, int d,
                                                   int L, FastPlan plan, uint8_t* __restrict__ frame_out,
                                                   double* __restrict__ idx_out, float* __restrict__ mm_out) {
  using Geo = FastGeo<NS>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  double* tree = reinterpret_cast<double*>(smem);
  uint32_t* lut = reinterpret_cast<uint32_t*>(smem + Geo::tree_len() * 8);
  uint8_t* frame = smem + Geo::frame_off();
  const int lane = threadIdx.x;
  for (int j = lane; j < Geo::G; j += 64) {
    uint32_t code = 0, off = 0;
    for (uint32_t m = 0; m < 4; ++m) {
      uint32_t x, y;
      d2xy(NS, 4 * j + m, x, y);
      if (m == 0) off = (y & ~1u) * NS + (x & ~1u);
      code |= ((x & 1u) + 2u * (y & 1u)) << (2 * m);
    }
    lut[j] = off | (code << 16);
  }
  // level-2 nodes of all-padding groups (t >= ND) are 0.0 for every embedding: zero once
  for (int k = lane; k < Geo::tree_len(); k += 64) tree[k] = 0.0;
  __syncthreads();

  const int slev = lane < L ? (int)plan.lev[lane] : -1;
  const int spos = lane < L ? plan.pos[lane] : 0;
  const bool pad0 = (d < NS * NS) || plan.zero_row;
  uint32_t lut_r[ND];  // loop-invariant: this lane's groups lane + 64 t
#pragma unroll
  for (int t = 0; t < ND; ++t) lut_r[t] = lut[lane + 64 * t];
  // V & 4: three register buffers — while embedding e is processed, e+G and e+2G are in flight (HBM
  // latency under full load is several microseconds; one embedding of prefetch left waves ~70%
  // stalled); otherwise two buffers.
  const int64_t G = gridDim.x;
  int64_t e = blockIdx.x;
  if constexpr ((V & 4) != 0) {
    Buf<NS, ND> A, B, C;
    if (e < N) load_emb<NS, ND, V>(in + e * stride, d, lane, slev, spos, A);
    if (e + G < N) load_emb<NS, ND, V>(in + (e + G) * stride, d, lane, slev, spos, B);
    while (e < N) {
      if (e + 2 * G < N) load_emb<NS, ND, V>(in + (e + 2 * G) * stride, d, lane, slev, spos, C);
      process_emb<NS, ND, V>(e, A, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out);
      e += G;
      if (e >= N) break;
      if (e + 2 * G < N) load_emb<NS, ND, V>(in + (e + 2 * G) * stride, d, lane, slev, spos, A);
      process_emb<NS, ND, V>(e, B, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out);
      e += G;
      if (e >= N) break;
      if (e + 2 * G < N) load_emb<NS, ND, V>(in + (e + 2 * G) * stride, d, lane, slev, spos, B);
      process_emb<NS, ND, V>(e, C, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out);
      e += G;
    }
  } else {
    Buf<NS, ND> A, B;
    if (e < N) load_emb<NS, ND, V>(in + e * stride, d, lane, slev, spos, A);
    while (e < N) {
      if (e + G < N) load_emb<NS, ND, V>(in + (e + G) * stride, d, lane, slev, spos, B);
      process_emb<NS, ND, V>(e, A, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out);
      e += G;
      if (e >= N) break;
      if (e + G < N) load_emb<NS, ND, V>(in + (e + G) * stride, d, lane, slev, spos, A);
      process_emb<NS, ND, V>(e, B, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out);
      e += G;
    }
  }
}

__device__ constexpr GroupLut<16> kLut16 = make_group_lut<16, false>();
__device__ constexpr GroupLut<32> kLut32 = make_group_lut<32, false>();
__device__ constexpr GroupLut<64> kLut64 = make_group_lut<64, false>();
template <int NS>
__device__ __forceinline__ const uint32_t* group_lut() {
  if constexpr (NS == 16) return kLut16.v;
  else if constexpr (NS == 32) return kLut32.v;
  else return kLut64.v;
}

// Non-persistent form (V & 64): one embedding per wave, WPB waves per workgroup, grid = N / WPB.  The
// hardware dispatcher interleaves the waves' streams; measured on the fused kernel's exact traffic
// shape (tools/ubench/hbm_shapes.hip) this moves 5.3 TB/s against 4.8-4.95 TB/s for every persistent
// grid-stride form.  Each wave owns a tree + frame slice of LDS; the per-lane LUT entries come from
// the compile-time table (L2 resident).
template <int NS>
struct NpGeo {
  static constexpr int tree_bytes = FastGeo<NS>::tree_len() * 8;
  static constexpr int frame_off = (tree_bytes + 15) & ~15;
  static constexpr int frame_bytes = (FastGeo<NS>::FB + 15) & ~15;
  static constexpr int wave_bytes = frame_off + frame_bytes;
  // V & 512: the frame overlays the tree (the tree is dead once the index slots are read), so a wave
  // needs max(tree, frame) bytes of LDS and more waves fit on a CU
  static constexpr int alias_bytes = frame_off > frame_bytes ? frame_off : frame_bytes;
};

template <int NS, int ND, int V, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_fused_np(const float* __restrict__ in, int64_t N, int64_t stride, int d,
                                                       int L, FastPlan plan, uint8_t* __restrict__ frame_out,
                                                       double* __restrict__ idx_out, float* __restrict__ mm_out) {
  using Geo = FastGeo<NS>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  constexpr bool kAlias = (V & 512) != 0;
  uint8_t* base = smem + wv * (kAlias ? NpGeo<NS>::alias_bytes : NpGeo<NS>::wave_bytes);
  double* tree = reinterpret_cast<double*>(base);
  uint8_t* frame = base + (kAlias ? 0 : NpGeo<NS>::frame_off);
  const int64_t e = (int64_t)blockIdx.x * WPB + wv;
  const bool live = e < N;
  const int slev = lane < L ? (int)plan.lev[lane] : -1;
  const int spos = lane < L ? plan.pos[lane] : 0;
  const bool pad0 = (d < NS * NS) || plan.zero_row;
  Buf<NS, ND> A;
  if (live) {
    load_emb<NS, ND, V>(in + e * stride, d, lane, slev, spos, A);
  } else {
#pragma unroll
    for (int t = 0; t < ND; ++t) A.g[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    A.slot = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // this lane's LUT entries (groups lane + 64 t), loaded alongside the embedding
  uint32_t lut_r[ND];
  const uint32_t* glut = group_lut<NS>();
#pragma unroll
  for (int t = 0; t < ND; ++t) lut_r[t] = glut[lane + 64 * t];
  // level-2 nodes of the all-padding groups t >= ND stay 0.0
  for (int k = 16 * ND + lane; k < Geo::G / 4; k += 64) tree[Geo::off(2) + k] = 0.0;
  process_emb<NS, ND, V>(e, A, d, L, lane, slev, spos, pad0, tree, lut_r, frame, frame_out, idx_out, mm_out, live);
}

template <int NS, int ND, int V>
static int launch_ff(const float* in, int64_t N, int64_t stride, int d, int L, const FastPlan& plan, uint8_t* frame,
                     double* idx, float* mm, hipStream_t s) {
  using Geo = FastGeo<NS>;
  const size_t lds = Geo::lds_bytes();
  const int grid = persistent_grid((const void*)k_fused_fast<NS, ND, V>, 64, lds, N);
  hipLaunchKernelGGL((k_fused_fast<NS, ND, V>), dim3(grid), dim3(64), lds, s, in, N, stride, d, L, plan, frame, idx,
                     mm);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int NS, int ND, int V>
static int launch_np(const float* in, int64_t N, int64_t stride, int d, int L, const FastPlan& plan, uint8_t* frame,
                     double* idx, float* mm, hipStream_t s) {
  constexpr int WPB = 1 << ((V >> 7) & 3);
  const size_t lds = (size_t)WPB * ((V & 512) ? NpGeo<NS>::alias_bytes : NpGeo<NS>::wave_bytes);
  const int64_t grid = (N + WPB - 1) / WPB;
  if (grid > 0x7FFFFFFF) return HQ_E_UNSUPPORTED;
  hipLaunchKernelGGL((k_fused_np<NS, ND, V, WPB>), dim3((unsigned)grid), dim3(64 * WPB), lds, s, in, N, stride, d, L,
                     plan, frame, idx, mm);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int NS, int ND, int V>
static int launch_any(const float* in, int64_t N, int64_t stride, int d, int L, const FastPlan& plan, uint8_t* frame,
                      double* idx, float* mm, hipStream_t s) {
  if constexpr ((V & 64) != 0) return launch_np<NS, ND, V>(in, N, stride, d, L, plan, frame, idx, mm, s);
  else return launch_ff<NS, ND, V>(in, N, stride, d, L, plan, frame, idx, mm, s);
}

// Variant bits (HQ_FUSED_V): 1 nt loads, 2 reciprocal quantize, 4 triple buffering (persistent), 8 / 16 / 32
// memory-only probes, 64 non-persistent (one embedding per wave), bits 7-8: log2 waves per workgroup,
// 512 frame overlays the tree in LDS (non-persistent form), 1024 / 2048 non-temporal frame / index stores
// (write-once outputs: +5% / +0.2%, tools/ab_fused.sh).
constexpr int kDefaultV = 64 | (1 << 7) | 512 | 1024 | 2048;  // non-persistent, 2 waves per workgroup, frame
                                                               // over tree, exact quantize, NT stores

template <int NS, int ND>
static int pick_nd(int variant, int nd, const float* in, int64_t N, int64_t stride, int d, int L, const FastPlan& plan,
                   uint8_t* frame, double* idx, float* mm, hipStream_t s) {
  if constexpr (ND > FastGeo<NS>::NT) {
    return HQ_E_UNSUPPORTED;
  } else {
    if (nd == ND) {
      if constexpr (NS == 64 && ND == 6) {  // A/B variants of the headline shape (HQ_FUSED_V, bench)
        switch (variant) {
          case 0: return launch_ff<NS, ND, 0>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 1: return launch_ff<NS, ND, 1>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 2: return launch_ff<NS, ND, 2>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 3: return launch_ff<NS, ND, 3>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 5: return launch_ff<NS, ND, 5>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 6: return launch_ff<NS, ND, 6>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 7: return launch_ff<NS, ND, 7>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 64: return launch_any<NS, ND, 64>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 192: return launch_any<NS, ND, 192>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 320: return launch_any<NS, ND, 320>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 448: return launch_any<NS, ND, 448>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 321: return launch_any<NS, ND, 321>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 322: return launch_any<NS, ND, 322>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 576: return launch_any<NS, ND, 576>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 704: return launch_any<NS, ND, 704>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 832: return launch_any<NS, ND, 832>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 960: return launch_any<NS, ND, 960>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 706: return launch_any<NS, ND, 706>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 1728: return launch_any<NS, ND, 1728>(in, N, stride, d, L, plan, frame, idx, mm, s);
#ifdef HQ_DIAG  // memory-only probes (bits 8 / 16 / 32): wrong outputs, A/B builds only (make DIAG=1)
          case 8: return launch_ff<NS, ND, 8>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 12: return launch_ff<NS, ND, 12>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 24: return launch_ff<NS, ND, 24>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 40: return launch_ff<NS, ND, 40>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 56: return launch_ff<NS, ND, 56>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 328: return launch_any<NS, ND, 328>(in, N, stride, d, L, plan, frame, idx, mm, s);
          case 840: return launch_any<NS, ND, 840>(in, N, stride, d, L, plan, frame, idx, mm, s);
#endif
          default: break;
        }
      }
      if (variant == 4) return launch_ff<NS, ND, 4>(in, N, stride, d, L, plan, frame, idx, mm, s);
      return launch_any<NS, ND, kDefaultV>(in, N, stride, d, L, plan, frame, idx, mm, s);
    }
    return pick_nd<NS, ND + 1>(variant, nd, in, N, stride, d, L, plan, frame, idx, mm, s);
  }
}

// Returns HQ_E_UNSUPPORTED (without launching) when the fast path does not apply.
int fused_fast(const float* in, int64_t N, int64_t stride, int d, int n, int L, uint8_t* frame, double* idx,
               float* mm, hipStream_t s) {
  if (!(n == 16 || n == 32 || n == 64)) return HQ_E_UNSUPPORTED;
  if (L < 1 || L > 64 || !idx || d < 1) return HQ_E_UNSUPPORTED;
  if ((reinterpret_cast<uintptr_t>(in) & 15) || (stride % 4) || (reinterpret_cast<uintptr_t>(frame) & 15) ||
      (reinterpret_cast<uintptr_t>(mm) & 7))
    return HQ_E_UNSUPPORTED;
  StreamSchedule sched;
  stream_schedule((int64_t)n * n, L, sched);
  FastPlan plan;
  plan.zero_row = 0;
  for (int i = 0; i < 64; ++i) {
    int lev = -1;
    int64_t pos = 0;
    if (i < L && stream_sample(sched, i, lev, pos)) {
      plan.lev[i] = (int8_t)lev;
      plan.pos[i] = (int32_t)pos;
    } else {
      plan.lev[i] = -1;
      plan.pos[i] = 0;
      if (i < n) plan.zero_row = 1;
    }
  }
  if (L < n) plan.zero_row = 1;
  const int nd = (((d + 3) / 4) + 63) / 64;
  const int variant = (int)opt(OPT_FUSED_V, kDefaultV);
  switch (n) {
    case 16: return pick_nd<16, 1>(variant, nd, in, N, stride, d, L, plan, frame, idx, mm, s);
    case 32: return pick_nd<32, 1>(variant, nd, in, N, stride, d, L, plan, frame, idx, mm, s);
    case 64: return pick_nd<64, 1>(variant, nd, in, N, stride, d, L, plan, frame, idx, mm, s);
  }
  return HQ_E_UNSUPPORTED;
}

}  // namespace hq
