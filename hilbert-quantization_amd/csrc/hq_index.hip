// hq_index.hip — block-mean index generators and the config-5 chunk
// encoder (f16 parameter stream -> per-1024-chunk traditional index + uint8 frame).
//
// References:
//   I2  core/index_generator.py:34-219,313-356 (traditional index, incl. the is_offset_sampling
//       quirk at :329-332 that turns every later level into corner/centre samples)
//   I4  rag/embedding_generation/hierarchical_index_generator.py:23-68,103-146,204-244,286-342
//   cfg5 core/streaming_processor.py:539-582 (1024-value chunks, astype(float32)) and :877-913
//       (encode_chunk: optimal dims, map_to_2d, traditional index with L = min(1024, n), embed,
//       compressor normalise)
//
// np.mean over a 2-D block is a pairwise sum over the C-order-flattened block in the image dtype
// (NumPy buffers the block contiguously), divided as f32(f64(sum) / count) for float32 — emulated
// exactly below so the index values are bit-identical.
#include "hq_common.h"

#include <stdlib.h>

namespace hq {

// np.mean over a (h x w) block with leading dimension ld, NumPy order (hq_common.h np_sum):
// f32 -> f32(f64(sum) / count) (numpy/_core/_methods.py _mean), f64 -> sum / count.
template <typename T>
__device__ __forceinline__ T np_mean_block(const T* b, int w, int ld, int h) {
  auto f = [=](int k) -> T { return b[(k / w) * ld + (k % w)]; };
  T s = np_sum<T>(f, w * h);
  if constexpr (sizeof(T) == 4) return (float)((double)s / (double)(w * h));
  else return s / (double)(w * h);
}

// ---------------------------------------------------------------------------------------------
// traditional index schedule (core/index_generator.py:34-98, 313-346)
// ---------------------------------------------------------------------------------------------
constexpr int kMaxAlloc = 16;
struct TradPlan {
  int cnt;
  int grid[kMaxAlloc];
  int alloc[kMaxAlloc];
  int sampling[kMaxAlloc];  // offset sampling (quirk) instead of block means
  int count[kMaxAlloc];     // values contributed
  int first[kMaxAlloc];     // first output slot
  int produced;
};

static void trad_plan(int n, int L, TradPlan& p) {
  p.cnt = 0;
  p.produced = 0;
  if (L <= 0) return;
  int gl[kMaxAlloc], al[kMaxAlloc], c = 0;
  int remaining = L;
  int max_grid = isqrt_floor(L);
  if (max_grid > 32) max_grid = 32;
  int g = 1;
  while (g <= max_grid) g *= 2;
  g /= 2;
  if (g < 2) g = 2;
  double frac = 0.5;
  while (remaining > 0 && g >= 1 && c < kMaxAlloc - 1) {
    int a = (int)((double)remaining * frac);
    if (g * g < a) a = g * g;
    if (remaining < a) a = remaining;
    if (a > 0) { gl[c] = g; al[c] = a; ++c; remaining -= a; }
    g /= 2;
    frac *= 0.5;
    if (frac < 0.01) break;
  }
  if (remaining > 0 && c > 0) { gl[c] = gl[0]; al[c] = remaining; ++c; }
  int out = 0;
  for (int i = 0; i < c; ++i) {
    bool in_prev = false;
    for (int k = 0; k < c - 1; ++k) in_prev |= (gl[k] == gl[i]);
    bool samp = (out > 0) && in_prev;
    int cnt;
    if (samp) {
      int sec = n / gl[i];
      if (sec < 1) sec = 1;
      int sy = n / sec;
      if (sy == 0) cnt = al[i] < 5 ? al[i] : 5;
      else {
        int ns = al[i] / 5;
        if (ns > sy * sy) ns = sy * sy;
        cnt = 5 * ns;
        if (cnt > al[i]) cnt = al[i];
      }
    } else {
      int sh = n / gl[i];
      int navg = (sh == 0) ? 1 : gl[i] * gl[i];
      cnt = navg < al[i] ? navg : al[i];
    }
    p.grid[i] = gl[i];
    p.alloc[i] = al[i];
    p.sampling[i] = samp;
    p.count[i] = cnt;
    p.first[i] = out;
    out += cnt;
  }
  p.cnt = c;
  p.produced = out;
}

// value of output slot i of the traditional index for an n x n f32 image with leading dim ld
__device__ float trad_slot(const float* img, int n, int ld, const TradPlan& p, int i) {
  if (i >= p.produced) return 0.f;
  for (int e = 0; e < p.cnt; ++e) {
    if (i >= p.first[e] + p.count[e]) continue;
    int k = i - p.first[e];
    int g = p.grid[e];
    if (!p.sampling[e]) {
      int sh = n / g;
      if (sh == 0) return np_mean_block(img, n, ld, n);
      int r = k / g, c = k % g;
      return np_mean_block(img + (r * sh) * ld + c * sh, sh, ld, sh);
    }
    int sec = n / g;
    if (sec < 1) sec = 1;
    int sy = n / sec;
    if (sy == 0) {
      const int h = n, w = n;
      switch (k) {
        case 0: return img[0];
        case 1: return img[w - 1];
        case 2: return img[(h - 1) * ld];
        case 3: return img[(h - 1) * ld + w - 1];
        default: return img[(h / 2) * ld + w / 2];
      }
    }
    int s = k / 5, which = k % 5;
    int r = s / sy, c = s % sy;  // sections visited row-major (sections_x == sections_y)
    int r0 = r * sec, r1 = r0 + sec, c0 = c * sec, c1 = c0 + sec;
    switch (which) {
      case 0: return img[r0 * ld + c0];
      case 1: return img[r0 * ld + c1 - 1];
      case 2: return img[(r1 - 1) * ld + c0];
      case 3: return img[(r1 - 1) * ld + c1 - 1];
      default: return img[((r0 + r1) / 2) * ld + (c0 + c1) / 2];
    }
  }
  return 0.f;
}

__global__ __launch_bounds__(64) void k_trad_image(const float* __restrict__ img, int64_t N, int n, int L,
                                                   TradPlan plan, float* __restrict__ out) {
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const float* im = img + e * (int64_t)n * n;
    for (int i = threadIdx.x; i < L; i += 64) out[e * (int64_t)L + i] = trad_slot(im, n, n, plan, i);
  }
}

// Host: image cell (row-major offset in an n x n image) that output slot i samples, -1 for a zero
// slot, -2 for a block-mean slot (same case analysis as trad_slot).
static int trad_cell(int n, const TradPlan& p, int i) {
  if (i >= p.produced) return -1;
  for (int e = 0; e < p.cnt; ++e) {
    if (i >= p.first[e] + p.count[e]) continue;
    const int k = i - p.first[e], g = p.grid[e];
    if (!p.sampling[e]) return -2;
    int sec = n / g;
    if (sec < 1) sec = 1;
    const int sy = n / sec;
    if (sy == 0) {
      const int h = n, w = n;
      const int cells[5] = {0, w - 1, (h - 1) * n, (h - 1) * n + w - 1, (h / 2) * n + w / 2};
      return cells[k < 4 ? k : 4];
    }
    const int sidx = k / 5, which = k % 5;
    const int r = sidx / sy, c = sidx % sy;
    const int r0 = r * sec, r1 = r0 + sec, c0 = c * sec, c1 = c0 + sec;
    const int cells[5] = {r0 * n + c0, r0 * n + c1 - 1, (r1 - 1) * n + c0, (r1 - 1) * n + c1 - 1,
                          ((r0 + r1) / 2) * n + (c0 + c1) / 2};
    return cells[which];
  }
  return -1;
}

// Slot plan of the fast chunk kernel: slots [0, fm) are 8 x 8 block means on a gm x gm block grid,
// slots [fm, n) read cell[i] (or 0.0 when cell[i] < 0).
struct ChunkPlan {
  int16_t cell[64];
  int fm, gm;
};

// ---------------------------------------------------------------------------------------------
// config 5: chunked f16 stream -> map -> traditional index -> embed -> uint8 frame
// one wave per chunk; image staged in LDS (f32, row-major)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float wmin(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t q8(float x, float mn, float rng) {
  float t = (x - mn) / rng;
  t = t * 255.0f;
  return (uint32_t)t;
}

template <int NS>
__global__ __launch_bounds__(64) void k_chunk(const __half* __restrict__ src, int64_t total, int chunk,
                                              int64_t c_begin, int64_t c_end, int L, TradPlan plan,
                                              uint8_t* __restrict__ frame_out, int64_t frame_stride,
                                              float* __restrict__ idx_out, int64_t idx_stride,
                                              float* __restrict__ mm_out) {
  constexpr int CELLS = NS * NS;
  constexpr int G = CELLS / 4;
  __shared__ __attribute__((aligned(16))) float img[CELLS];
  __shared__ uint32_t lut[G];
  __shared__ float rowv[NS];
  const int lane = threadIdx.x;
  for (int j = lane; j < G; j += 64) {
    uint32_t code = 0, off = 0;
    for (uint32_t m = 0; m < 4; ++m) {
      uint32_t x, y;
      d2xy(NS, 4 * j + m, x, y);
      if (m == 0) off = (y & ~1u) * NS + (x & ~1u);
      code |= m << (2 * ((x & 1u) + 2u * (y & 1u)));  // inverse: slot b holds element m
    }
    lut[j] = off | (code << 16);
  }
  __syncthreads();
  for (int64_t c = c_begin + blockIdx.x; c < c_end; c += gridDim.x) {
    const int64_t base = c * (int64_t)chunk;
    int64_t cnt64 = total - base;
    const int cnt = (int)(cnt64 < chunk ? cnt64 : chunk);
    const __half* s = src + base;
    float lmin = __builtin_huge_valf(), lmax = -__builtin_huge_valf();
    for (int j = lane; j < G; j += 64) {
      float v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        int i = 4 * j + m;
        v[m] = (i < cnt) ? __half2float(s[i]) : 0.f;
        if (i < cnt) { lmin = fminf(lmin, v[m]); lmax = fmaxf(lmax, v[m]); }
      }
      uint32_t ent = lut[j], off = ent & 0xFFFFu, code = ent >> 16;
      float a0 = v[(code >> 0) & 3], a1 = v[(code >> 2) & 3], a2 = v[(code >> 4) & 3], a3 = v[(code >> 6) & 3];
      *reinterpret_cast<float2*>(img + off) = make_float2(a0, a1);
      *reinterpret_cast<float2*>(img + off + NS) = make_float2(a2, a3);
    }
    float mn = wmin(lmin), mx = wmax(lmax);
    if (cnt < CELLS) { mn = fminf(mn, 0.f); mx = fmaxf(mx, 0.f); }
    __syncthreads();
    float rmin = __builtin_huge_valf(), rmax = -__builtin_huge_valf();
    for (int i = lane; i < NS; i += 64) {
      float v = (i < L) ? trad_slot(img, NS, NS, plan, i) : 0.f;
      rowv[i] = v;
      rmin = fminf(rmin, v);
      rmax = fmaxf(rmax, v);
    }
    for (int i = lane; i < L; i += 64)
      idx_out[c * idx_stride + i] = (i < NS) ? rowv[i] : trad_slot(img, NS, NS, plan, i);
    mn = fminf(mn, wmin(rmin));
    mx = fmaxf(mx, wmax(rmax));
    const bool flat = mx == mn;
    const float rng = mx - mn;
    uint8_t* dst = frame_out + c * frame_stride;
    // body: 16 cells per lane per step, 16-byte stores
    for (int q = lane; q < CELLS / 16; q += 64) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float4 f = *reinterpret_cast<const float4*>(img + 16 * q + 4 * k);
        if (flat) {
          w[k] = 0x80808080u;
        } else {
          w[k] = q8(f.x, mn, rng) | (q8(f.y, mn, rng) << 8) | (q8(f.z, mn, rng) << 16) | (q8(f.w, mn, rng) << 24);
        }
      }
      *reinterpret_cast<uint4*>(dst + 16 * q) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (CELLS < 16)
      for (int q = lane; q < CELLS; q += 64) dst[q] = flat ? 128 : (uint8_t)q8(img[q], mn, rng);
    for (int i = lane; i < NS; i += 64) dst[CELLS + i] = flat ? 128 : (uint8_t)q8(rowv[i], mn, rng);
    if (lane == 0) { mm_out[2 * c] = mn; mm_out[2 * c + 1] = mx; }
    __syncthreads();
  }
}

// Fast form for whole chunks of exactly NS x NS values (cfg5: 1024 -> 32 x 32): one chunk per wave,
// WPB waves per workgroup, no persistent loop (the non-persistent shape streams ~10% faster on this
// chip, tools/ubench/hbm_shapes.hip).  Each lane loads 16-byte runs of the f16 stream (two float4
// groups = two 2x2 image blocks) and scatters them into the wave's LDS image with the compile-time
// group LUT; the traditional index and the 16-byte frame stores follow k_chunk.
__device__ constexpr AddrLut<32> kAddr32 = make_addr_lut<32>();
__device__ constexpr AddrLut<64> kAddr64 = make_addr_lut<64>();

__device__ __forceinline__ float2 h2f(uint32_t w) {
  return make_float2(__half2float(__ushort_as_half((unsigned short)(w & 0xFFFFu))),
                     __half2float(__ushort_as_half((unsigned short)(w >> 16))));
}

// NT: non-temporal stores of the write-once outputs (frames, index rows, min/max)
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int NS, int WPB, bool FQ, int CPW, int NT>
__global__ __launch_bounds__(64 * WPB) void k_chunk_np(const uint16_t* __restrict__ src, int64_t nchunks,
                                                       ChunkPlan plan, uint8_t* __restrict__ frame_out,
                                                       float* __restrict__ idx_out, float* __restrict__ mm_out) {
  constexpr int CELLS = NS * NS;
  constexpr int NU = CELLS / 512;  // 16-byte loads per lane (8 values = two groups)
  constexpr int FB = (NS + 1) * NS;
  __shared__ __attribute__((aligned(16))) float img_all[WPB][CELLS];
  __shared__ float rowv_all[WPB][NS];
  __shared__ __attribute__((aligned(16))) uint8_t rowq_all[WPB][NS];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  float* img = img_all[wv];
  float* rowv = rowv_all[wv];
  const int64_t c0 = ((int64_t)blockIdx.x * WPB + wv) * CPW;
  const uint32_t* alut = NS == 32 ? kAddr32.v : kAddr64.v;
  // CPW chunks per wave, all loaded up front (more bytes in flight per wave)
  uint4 raw_all[CPW][NU];
  uint32_t ent[4 * NU];  // LDS byte offsets of the lane's 8 NU values, two per dword (AddrLut)
#pragma unroll
  for (int k = 0; k < CPW; ++k)
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if constexpr ((NT & 2) != 0) {  // non-temporal loads (A/B)
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        const u4v r = c0 + k < nchunks
                          ? __builtin_nontemporal_load(reinterpret_cast<const u4v*>(src + (c0 + k) * CELLS) + lane + 64 * u)
                          : u4v{0u, 0u, 0u, 0u};
        raw_all[k][u] = make_uint4(r.x, r.y, r.z, r.w);
      } else {
        raw_all[k][u] = c0 + k < nchunks ? reinterpret_cast<const uint4*>(src + (c0 + k) * CELLS)[lane + 64 * u]
                                         : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const uint4 e = reinterpret_cast<const uint4*>(alut)[lane + 64 * u];  // values 8 (lane + 64 u) ..
    ent[4 * u] = e.x;
    ent[4 * u + 1] = e.y;
    ent[4 * u + 2] = e.z;
    ent[4 * u + 3] = e.w;
  }
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
  const int64_t c = c0 + k;
  const bool live = c < nchunks;
  if (WPB == 1 && !live) break;
  const uint4* raw = raw_all[k];
  float lmin = __builtin_huge_valf(), lmax = -__builtin_huge_valf();
#pragma unroll
  for (int u = 0; u < NU; ++u) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float2 a = h2f(h ? raw[u].z : raw[u].x), b = h2f(h ? raw[u].w : raw[u].y);
      lmin = fminf(lmin, fminf(fminf(a.x, a.y), fminf(b.x, b.y)));
      lmax = fmaxf(lmax, fmaxf(fmaxf(a.x, a.y), fmaxf(b.x, b.y)));
      // four b32 LDS stores at the group's precomputed byte offsets (one mask or shift each)
      const uint32_t e0 = ent[4 * u + 2 * h], e1 = ent[4 * u + 2 * h + 1];
      auto at = [&](uint32_t byte_off) { return reinterpret_cast<float*>(reinterpret_cast<char*>(img) + byte_off); };
      *at(e0 & 0xFFFFu) = a.x;
      *at(e0 >> 16) = a.y;
      *at(e1 & 0xFFFFu) = b.x;
      *at(e1 >> 16) = b.y;
    }
  }
  __syncthreads();
  // first-level block means (slots < fm, 8 x 8 blocks in row-major block order): np.mean's pairwise
  // order for 64 values is eight column accumulators r_j (rows in order), then
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)); four lanes per block hold two columns each and combine by
  // xor-1 / xor-2 exchanges (IEEE addition is commutative, so both partners get the same bits).
  constexpr int gm = NS / 8;  // the fast form runs only when the first level is NS/8 x NS/8 blocks of 8 x 8
  const int fm = plan.fm;
  for (int r = 0; r < (fm + 15) / 16; ++r) {
    const int b = (lane >> 2) + 16 * r, q = lane & 3;
    const int bb = b < fm ? b : 0;
    const float* blk = img + ((bb / gm) * 8) * NS + (bb % gm) * 8 + 2 * q;
    float2 acc = *reinterpret_cast<const float2*>(blk);
#pragma unroll
    for (int row = 1; row < 8; ++row) {
      const float2 v = *reinterpret_cast<const float2*>(blk + row * NS);
      acc.x = acc.x + v.x;
      acc.y = acc.y + v.y;
    }
    float t = acc.x + acc.y;
    t = t + dppf<0xB1>(t);  // quad_perm xor 1
    t = t + dppf<0x4E>(t);  // quad_perm xor 2
    t = 0.0f + t;
    if (q == 0 && b < fm) rowv[b] = (float)((double)t / 64.0);
  }
  if (lane >= fm && lane < NS) {
    const int cell = plan.cell[lane];
    rowv[lane] = cell >= 0 ? img[cell] : 0.0f;
  }
  __syncthreads();
  if (lane < NS) {
    const float iv = rowv[lane];
    lmin = fminf(lmin, iv);
    lmax = fmaxf(lmax, iv);
    if (live) st_out(idx_out + c * NS + lane, iv, (NT & 1) != 0);
  }
  const float mn = wmin64(lmin), mx = wmax64(lmax);
  if (live) {
  const bool flat = mx == mn;
  const float rng = mx - mn;
  // hardware reciprocal (1 ulp; the fast form's bound with it: qfast, hq_common.h); f16 data gives
  // rng >= 2^-24 or a flat frame, so 1 / rng stays finite
  const float rcp = __builtin_amdgcn_rcpf(rng);
  uint8_t* dst = frame_out + c * FB;
  // one quantized byte: reciprocal form with an exact fallback per cell position (qfast, hq_common.h)
  // — the IEEE division runs only where some lane's value lies within 1e-3 of a level edge
  auto qb = [&](float x) -> uint32_t {
    if constexpr (FQ) {
      bool slow = false;
      uint32_t v = qfast(x, mn, rcp, slow);
      if (__builtin_amdgcn_ballot_w64(slow))
        if (slow) v = q8(x, mn, rng);
      return v;
    } else {
      return q8(x, mn, rng);
    }
  };
  // image body: 16 cells per lane, 16-byte stores.  Fast form as packed f32 over cell pairs:
  // y = (x - mn) * fl(fl(1/rng) * 255) (five roundings in all, the same < 7.7e-5 bound as qfast),
  // byte = floor(y) packed with v_cvt_pk_u8_f32 (exact: an integer <= 255), and the exact division
  // redone at a cell position only where some lane has |frac(y) - 0.5| > 0.4999.
  typedef float f2v __attribute__((ext_vector_type(2)));
  const float c255 = rcp * 255.0f;
  const f2v mn2 = {mn, mn}, c2 = {c255, c255}, h2 = {0.5f, 0.5f};
#pragma unroll
  for (int q = lane; q < CELLS / 16; q += 64) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 f = *reinterpret_cast<const float4*>(img + 16 * q + 4 * k);
      if (flat) {
        w[k] = 0x80808080u;
      } else if constexpr (FQ) {
        const f2v ya = (f2v{f.x, f.y} - mn2) * c2, yb = (f2v{f.z, f.w} - mn2) * c2;
        const f2v fa = {floorf(ya.x), floorf(ya.y)}, fb = {floorf(yb.x), floorf(yb.y)};
        const f2v ta = (ya - fa) - h2, tb = (yb - fb) - h2;
        uint32_t word = __builtin_amdgcn_cvt_pk_u8_f32(fa.x, 0, 0u);
        word = __builtin_amdgcn_cvt_pk_u8_f32(fa.y, 1, word);
        word = __builtin_amdgcn_cvt_pk_u8_f32(fb.x, 2, word);
        word = __builtin_amdgcn_cvt_pk_u8_f32(fb.y, 3, word);
        const float xs[4] = {f.x, f.y, f.z, f.w};
        const bool sl[4] = {fabsf(ta.x) > 0.4999f, fabsf(ta.y) > 0.4999f, fabsf(tb.x) > 0.4999f, fabsf(tb.y) > 0.4999f};
        if (__builtin_amdgcn_ballot_w64(sl[0] | sl[1] | sl[2] | sl[3]))  // one branch per four cells
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (__builtin_amdgcn_ballot_w64(sl[m]))
              if (sl[m]) word = (word & ~(0xFFu << (8 * m))) | (q8(xs[m], mn, rng) << (8 * m));
        w[k] = word;
      } else {
        w[k] = qb(f.x) | (qb(f.y) << 8) | (qb(f.z) << 16) | (qb(f.w) << 24);
      }
    }
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    st_out(reinterpret_cast<u4v*>(dst + 16 * q), u4v{w[0], w[1], w[2], w[3]}, (NT & 1) != 0);
  }
  // index row: one value per lane, bytes packed through LDS (rowv's own slot), 16-byte stores
  uint8_t* rowq = rowq_all[wv];
  if (lane < NS) rowq[lane] = flat ? (uint8_t)128 : (uint8_t)qb(rowv[lane]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < NS / 16) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    st_out(reinterpret_cast<u4v*>(dst + CELLS + 16 * lane), reinterpret_cast<const u4v*>(rowq)[lane], (NT & 1) != 0);
  }
  if (lane == 0) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    st_out(reinterpret_cast<f2v*>(mm_out + 2 * c), f2v{mn, mx}, (NT & 1) != 0);
  }
  }
  if constexpr (CPW > 1) __syncthreads();  // the next chunk reuses the LDS image
  }
}

// ---------------------------------------------------------------------------------------------
// I4: RAG multi-row index
// ---------------------------------------------------------------------------------------------
static int rag_grans(int width, int* out) {
  int g = isqrt_floor(width);
  if (g < 2) g = 2;
  int p = 1;
  while (p * 2 <= g) p *= 2;
  int k = 0;
  for (int cur = p; cur >= 2 && k < 8; cur /= 2) out[k++] = cur;
  return k;
}

template <typename T>
__global__ __launch_bounds__(256) void k_rag(const T* __restrict__ img, int64_t N, int n, int R, int4 g03, int4 g47,
                                             T* __restrict__ out) {
  int grans[8] = {g03.x, g03.y, g03.z, g03.w, g47.x, g47.y, g47.z, g47.w};
  const int64_t cells = (int64_t)n * n;
  const int64_t ocells = (int64_t)(n + R) * n;
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const T* im = img + e * cells;
    T* o = out + e * ocells;
    for (int64_t c = threadIdx.x; c < cells; c += blockDim.x) o[c] = im[c];
    for (int c = threadIdx.x; c < R * n; c += blockDim.x) {
      int r = c / n, k = c % n;
      int g = grans[r];
      T val = T(0);
      if (k < g * g) {
        int sh = n / g;
        if (sh == 0) {
          val = np_mean_block(im, n, n, n);
        } else {
          uint32_t row, col;
          if (g == 2) {
            // hard-coded list (hierarchical_index_generator.py:302-303): (0,0),(0,1),(1,1),(1,0)
            const uint32_t rr[4] = {0, 0, 1, 1}, cc[4] = {0, 1, 1, 0};
            row = rr[k]; col = cc[k];
          } else {
            uint32_t x, y;
            d2xy(g, k, x, y);  // (row, col) order of the RAG generator == (y, x) of the core curve
            row = y; col = x;
          }
          val = np_mean_block(im + (row * sh) * n + col * sh, sh, n, sh);
        }
      }
      o[cells + c] = val;
    }
  }
}

static int optimal_side(int64_t count) {
  // core/dimension_calculator.py:36-61,105-128
  static const int64_t valid[] = {4, 16, 64, 256, 1024, 4096, 16384};
  int64_t size = -1;
  for (int64_t v : valid)
    if (v >= count) { size = v; break; }
  if (size < 0) { size = 16384; while (size < count) size *= 4; }
  int64_t s = 1;
  while (s * s < size) ++s;
  return (int)s;
}

// fast chunk kernel launch; HQ_E_UNSUPPORTED (nothing launched) when the slot plan does not fit it
template <int NS, int WPB, int CPW = 1>
static int launch_chunk_np(const uint16_t* in, int64_t nchunks, const TradPlan& plan, uint8_t* frame, float* idx,
                           float* mm, hipStream_t s) {
  const int64_t grid = (nchunks + WPB * CPW - 1) / (WPB * CPW);
  if (grid > 0x7FFFFFFF) return HQ_E_UNSUPPORTED;
  // slots [0, fm): first-level 8 x 8 block means (the only non-sampled level, index_generator.py:329-332);
  // every later slot must be a sample or a zero, else the generic kernel runs
  ChunkPlan cp{};
  cp.fm = 0;
  cp.gm = plan.cnt > 0 ? plan.grid[0] : 1;
  if (plan.cnt > 0 && !plan.sampling[0] && plan.first[0] == 0 && plan.grid[0] > 0 && NS / plan.grid[0] == 8)
    cp.fm = plan.count[0] < NS ? plan.count[0] : NS;
  for (int i = 0; i < 64; ++i) {
    const int cell = i < NS && i >= cp.fm ? trad_cell(NS, plan, i) : -1;
    if (cell == -2) return HQ_E_UNSUPPORTED;
    cp.cell[i] = (int16_t)cell;
  }
  const int nt = (int)opt(OPT_CHUNK_NT, 0);  // A/B bits: 1 non-temporal stores (measured equal), 2 loads
  if (opt_on(OPT_CHUNK_EXACTDIV))
    hipLaunchKernelGGL((k_chunk_np<NS, WPB, false, CPW, 0>), dim3((unsigned)grid), dim3(64 * WPB), 0, s, in,
                       nchunks, cp, frame, idx, mm);
  else if (nt == 1)
    hipLaunchKernelGGL((k_chunk_np<NS, WPB, true, CPW, 1>), dim3((unsigned)grid), dim3(64 * WPB), 0, s, in,
                       nchunks, cp, frame, idx, mm);
  else if (nt == 2)
    hipLaunchKernelGGL((k_chunk_np<NS, WPB, true, CPW, 2>), dim3((unsigned)grid), dim3(64 * WPB), 0, s, in,
                       nchunks, cp, frame, idx, mm);
  else if (nt == 3)
    hipLaunchKernelGGL((k_chunk_np<NS, WPB, true, CPW, 3>), dim3((unsigned)grid), dim3(64 * WPB), 0, s, in,
                       nchunks, cp, frame, idx, mm);
  else
    hipLaunchKernelGGL((k_chunk_np<NS, WPB, true, CPW, 0>), dim3((unsigned)grid), dim3(64 * WPB), 0, s, in,
                       nchunks, cp, frame, idx, mm);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int NS>
static int launch_chunk(const uint16_t* in, int64_t total, int chunk, int64_t c0, int64_t c1, uint8_t* frame,
                        int64_t fstride, float* idx, int64_t istride, float* mm, hipStream_t s) {
  int L = NS;  // min(1024, n) (core/streaming_processor.py:897-899)
  TradPlan plan;
  trad_plan(NS, L, plan);
  if constexpr (NS == 32 || NS == 64) {
    const bool aligned = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(frame)) & 15) == 0 &&
                         (reinterpret_cast<uintptr_t>(mm) & 7) == 0;
    if (chunk == NS * NS && c0 == 0 && fstride == (int64_t)(NS + 1) * NS && istride == NS && aligned &&
        !opt_on(OPT_CHUNK_GENERIC)) {
      // launch form (options chunk_wpb: waves per workgroup, chunk_cpw: chunks per wave)
      const int wpb = (int)opt(OPT_CHUNK_WPB, 1), cpw = (int)opt(OPT_CHUNK_CPW, 2);
      int rc;
      if (wpb == 2) rc = launch_chunk_np<NS, 2>(in, c1, plan, frame, idx, mm, s);
      else if (wpb == 4) rc = launch_chunk_np<NS, 4>(in, c1, plan, frame, idx, mm, s);
      else if (cpw == 4) rc = launch_chunk_np<NS, 1, 4>(in, c1, plan, frame, idx, mm, s);
      else if (cpw == 2) rc = launch_chunk_np<NS, 1, 2>(in, c1, plan, frame, idx, mm, s);
      else rc = launch_chunk_np<NS, 1, 1>(in, c1, plan, frame, idx, mm, s);
      if (rc != HQ_E_UNSUPPORTED) return rc;
    }
  }
  int grid = persistent_grid((const void*)k_chunk<NS>, 64, 0, c1 - c0);
  hipLaunchKernelGGL(k_chunk<NS>, dim3(grid), dim3(64), 0, s, (const __half*)in, total, chunk, c0, c1, L, plan,
                     frame, fstride, idx, istride, mm);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

static int dispatch_chunk(int ns, const uint16_t* in, int64_t total, int chunk, int64_t c0, int64_t c1,
                          uint8_t* frame, int64_t fstride, float* idx, int64_t istride, float* mm, hipStream_t s) {
  switch (ns) {
    case 2: return launch_chunk<2>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
    case 4: return launch_chunk<4>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
    case 8: return launch_chunk<8>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
    case 16: return launch_chunk<16>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
    case 32: return launch_chunk<32>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
    case 64: return launch_chunk<64>(in, total, chunk, c0, c1, frame, fstride, idx, istride, mm, s);
  }
  return fail(HQ_E_UNSUPPORTED, "chunk side %d (chunk encoder supports chunks of <= 4096 values)", ns);
}


// block means in row-major section order (core/index_generator.py:100-144) or in the RAG
// generator's Hilbert order (hierarchical_index_generator.py:204-244); one thread per block
template <typename T>
__global__ __launch_bounds__(256) void k_block_means(const T* __restrict__ img, int64_t N, int n, int g,
                                                     int order, T* __restrict__ out) {
  const int sh = n / g;
  const int cnt = sh == 0 ? 1 : g * g;
  const int64_t total = N * cnt;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / cnt;
    const int k = (int)(t % cnt);
    const T* im = img + e * (int64_t)n * n;
    T v;
    if (sh == 0) {
      v = np_mean_block(im, n, n, n);
    } else {
      uint32_t row, col;
      if (order == 0) {
        row = k / g; col = k % g;
      } else if (g == 2) {
        const uint32_t rr[4] = {0, 0, 1, 1}, cc[4] = {0, 1, 1, 0};
        row = rr[k]; col = cc[k];
      } else if (g == 1) {
        row = 0; col = 0;
      } else {
        uint32_t x, y;
        d2xy(g, k, x, y);
        row = y; col = x;
      }
      v = np_mean_block(im + (row * sh) * n + col * sh, sh, n, sh);
    }
    out[t] = v;
  }
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_index_traditional_f32(const float* img, int64_t N, int n, int L, float* out, hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Dimension must be a power of 2, got %d", n);
  if (N < 0 || L < 0) return fail(HQ_E_INVALID, "bad shape");
  if (N == 0 || L == 0) return HQ_OK;
  if (!img || !out) return fail(HQ_E_INVALID, "null buffer");
  TradPlan plan;
  trad_plan(n, L, plan);
  int grid = persistent_grid((const void*)k_trad_image, 64, 0, N);
  hipLaunchKernelGGL(k_trad_image, dim3(grid), dim3(64), 0, (hipStream_t)stream, img, N, n, L, plan, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_block_means(int dtype, const void* img, int64_t N, int n, int grid, int order, void* out,
                   hq_stream_t stream) {
  if (n <= 0 || grid <= 0 || N < 0) return fail(HQ_E_INVALID, "bad shape n=%d grid=%d", n, grid);
  if (N == 0) return HQ_OK;
  if (!img || !out) return fail(HQ_E_INVALID, "null buffer");
  const int cnt = (n / grid == 0) ? 1 : grid * grid;
  int64_t blocks = (N * cnt + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (dtype == HQ_F32)
    hipLaunchKernelGGL(k_block_means<float>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const float*)img, N,
                       n, grid, order, (float*)out);
  else if (dtype == HQ_F64)
    hipLaunchKernelGGL(k_block_means<double>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const double*)img,
                       N, n, grid, order, (double*)out);
  else
    return fail(HQ_E_UNSUPPORTED, "block means dtype %d (f32/f64)", dtype);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_rag_index_rows(int n) {
  int g[8];
  return rag_grans(n, g);
}

int hq_index_rag_f32(const float* img, int64_t N, int n, float* out, hq_stream_t stream) {
  if (n <= 0) return fail(HQ_E_INVALID, "bad width %d", n);
  if (N < 0) return fail(HQ_E_INVALID, "bad shape");
  if (N == 0) return HQ_OK;
  if (!img || !out) return fail(HQ_E_INVALID, "null buffer");
  int g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int R = rag_grans(n, g);
  int grid = persistent_grid((const void*)k_rag<float>, 256, 0, N);
  hipLaunchKernelGGL(k_rag<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, img, N, n, R,
                     make_int4(g[0], g[1], g[2], g[3]), make_int4(g[4], g[5], g[6], g[7]), out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_chunk_encode_f16(const uint16_t* in, int64_t total, int chunk, uint8_t* frame, float* idx, float* minmax,
                        hq_stream_t stream) {
  if (total < 0 || chunk <= 0) return fail(HQ_E_INVALID, "bad sizes total=%lld chunk=%d", (long long)total, chunk);
  if (total == 0) return HQ_OK;
  if (!in || !frame || !idx || !minmax) return fail(HQ_E_INVALID, "null buffer");
  const int ns = optimal_side(chunk);
  const int64_t nchunks = (total + chunk - 1) / chunk;
  const int64_t fstride = (int64_t)(ns + 1) * ns;
  const int64_t istride = ns;
  if ((fstride % 16) != 0 && ns >= 4) return fail(HQ_E_UNSUPPORTED, "frame stride %lld", (long long)fstride);
  hipStream_t s = (hipStream_t)stream;
  const int64_t tail = total % chunk;
  const int64_t full = tail ? nchunks - 1 : nchunks;
  if (full > 0) {
    int rc = dispatch_chunk(ns, in, total, chunk, 0, full, frame, fstride, idx, istride, minmax, s);
    if (rc) return rc;
  }
  if (tail) {
    const int ts = optimal_side(tail);
    // the tail chunk gets its own geometry ((ts+1) x ts frame, L = ts) inside the last slot;
    // launched with `chunk` so chunk index nchunks-1 addresses the right source offset
    uint8_t* f = frame + (nchunks - 1) * fstride;
    float* ix = idx + (nchunks - 1) * istride;
    float* m = minmax + 2 * (nchunks - 1);
    int rc = dispatch_chunk(ts, in + (nchunks - 1) * (int64_t)chunk, tail, chunk, 0, 1, f, 0, ix, 0, m, s);
    if (rc) return rc;
  }
  return HQ_OK;
}

}  // extern "C"
