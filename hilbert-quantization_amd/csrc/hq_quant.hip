// hq_quant.hip — the north-star kernel: fused Hilbert map + streaming hierarchical index +
// index-row embed + uint8 quantize, plus the standalone
// streaming-index (I1), quantize (Q1) and de-normalise (Q2) entry points.
//
// Reference sequence replaced (core/pipeline.py:97-146):
//   pad with 0.0 (:325-349) -> map_to_2d (core/hilbert_mapper.py:115-174)
//   -> StreamingHilbertIndexGenerator.generate_optimized_indices (core/streaming_index_builder.py:
//      315-343: 4-ary float64 mean tree over the Hilbert-ordered stream, per-level strided samples)
//   -> embed_indices_in_image (core/index_generator.py:221-253: index row cast to f32)
//   -> _normalize_for_compression (core/compressor.py:256-280: f32 min/max -> trunc(.. * 255))
//
// MI355X design (HBM-bound, 10,824 algorithmic bytes per 1536-d embedding):
//   * one wave64 workgroup per embedding, persistent grid-stride over embeddings;
//   * lane j reads float4 group j (stream elements 4j..4j+3) -> every global load is a coalesced
//     1 KiB wave instruction; the groups stay in registers for the second pass (n <= 64);
//   * level 1 of the mean tree is formed in registers (a group of 4 IS a tree node), levels >= 2
//     are LDS reductions in the reference's left-to-right f64 association order;
//   * a 2x2 block of the image is exactly one float4 group (Hilbert layout invariant), so each
//     lane quantizes its group and writes two u16 pairs into a row-major LDS frame; the frame is
//     then streamed to HBM with 16-byte stores — no scattered global writes;
//   * f32 quantize uses IEEE division (-ffp-contract=off, no fast-math) => bit-exact frames.
#include "hq_common.h"

#include <stdlib.h>

namespace hq {

__device__ __forceinline__ float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// reference quantize: ((x - mn) / (mx - mn) * 255).astype(uint8), all in float32
__device__ __forceinline__ uint32_t quant1(float x, float mn, float rng) {
  float t = (x - mn) / rng;
  t = t * 255.0f;
  return (uint32_t)t;
}

template <int NS>
struct FusedGeom {
  static constexpr int G = NS * NS / 4;             // float4 groups = 2x2 blocks
  static constexpr int NT = (G + 63) / 64;          // groups per lane
  static constexpr bool KEEP = NT <= 16;            // keep groups in registers for pass 2
  static constexpr int FB = (NS + 1) * NS;          // frame bytes
  static constexpr int FB16 = (FB + 15) & ~15;
  static constexpr int levels() {                   // stream levels (<= 10)
    int k = 0, s = NS * NS;
    while (k < kStreamMaxLevels && s > 0) { ++k; s >>= 2; }
    return k;
  }
  static constexpr int tree_len() {                 // f64 values of levels 1..levels-1
    int t = 0, s = G;
    for (int l = 1; l < levels(); ++l) { t += s; s >>= 2; }
    return t;
  }
  static constexpr int lvl_off(int l) {             // offset of level l (>= 1) in the tree
    int t = 0, s = G;
    for (int k = 1; k < l; ++k) { t += s; s >>= 2; }
    return t;
  }
  static constexpr size_t lds_bytes() {
    return (size_t)tree_len() * 8 + (size_t)G * 4 + FB16 + 16;
  }
};

// LUT entry for group j: byte offset of the 2x2 block's top-left pixel (row-major, bits 0..15) and
// for each element m the byte position b_m = dx + 2*dy inside [row0 lo, row0 hi, row1 lo, row1 hi]
// (bits 16 + 2m).
__device__ __forceinline__ uint32_t group_lut(uint32_t n, uint32_t j) {
  uint32_t code = 0, off = 0;
  for (uint32_t m = 0; m < 4; ++m) {
    uint32_t x, y;
    d2xy(n, 4 * j + m, x, y);
    if (m == 0) off = (y & ~1u) * n + (x & ~1u);
    code |= ((x & 1u) + 2u * (y & 1u)) << (2 * m);
  }
  return off | (code << 16);
}

template <int NS>
__global__ __launch_bounds__(64) void k_fused(const float* __restrict__ in, int64_t N, int64_t stride,
                                              int d, int L, bool vec_ok, StreamSchedule sched,
                                              uint8_t* __restrict__ frame_out, double* __restrict__ idx_out,
                                              float* __restrict__ minmax_out) {
  using Geo = FusedGeom<NS>;
  constexpr int G = Geo::G;
  constexpr int NT = Geo::NT;
  constexpr int NLEV = Geo::levels();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  double* tree = reinterpret_cast<double*>(smem);
  uint32_t* lut = reinterpret_cast<uint32_t*>(smem + Geo::tree_len() * 8);
  uint8_t* frame = smem + Geo::tree_len() * 8 + G * 4;
  frame = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(frame) + 15) & ~uintptr_t(15));
  const int lane = threadIdx.x;

  for (int j = lane; j < G; j += 64) lut[j] = group_lut(NS, j);
  __syncthreads();

  const int groups_data = (d + 3) / 4;  // groups holding at least one real element
  const bool padded = d < NS * NS;

  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const float* src = in + e * stride;
    float4 v[Geo::KEEP ? NT : 1];
    float lmin = __builtin_huge_valf(), lmax = -__builtin_huge_valf();

    // ---- pass 1: load, min/max, tree level 1 -------------------------------------------------
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int j = lane + 64 * t;
      if (j < G) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < groups_data) {
          if (vec_ok && 4 * j + 3 < d) {
            x = *reinterpret_cast<const float4*>(src + 4 * j);
          } else {
            if (4 * j + 0 < d) x.x = src[4 * j + 0];
            if (4 * j + 1 < d) x.y = src[4 * j + 1];
            if (4 * j + 2 < d) x.z = src[4 * j + 2];
            if (4 * j + 3 < d) x.w = src[4 * j + 3];
          }
          if (4 * j + 3 < d) {
            lmin = fminf(lmin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
            lmax = fmaxf(lmax, fmaxf(fmaxf(x.x, x.y), fmaxf(x.z, x.w)));
          } else {
            if (4 * j + 0 < d) { lmin = fminf(lmin, x.x); lmax = fmaxf(lmax, x.x); }
            if (4 * j + 1 < d) { lmin = fminf(lmin, x.y); lmax = fmaxf(lmax, x.y); }
            if (4 * j + 2 < d) { lmin = fminf(lmin, x.z); lmax = fmaxf(lmax, x.z); }
          }
        }
        if constexpr (Geo::KEEP) v[t] = x;
        if (NLEV > 1) {
          // (window[0] + window[1] + window[2] + window[3]) * 0.25 in double (:96)
          double s = (((double)x.x + (double)x.y) + (double)x.z) + (double)x.w;
          tree[j] = s * 0.25;
        }
      }
    }
    float mn = wave_min(lmin), mx = wave_max(lmax);
    if (padded) { mn = fminf(mn, 0.f); mx = fmaxf(mx, 0.f); }
    __syncthreads();

    // ---- tree levels >= 2 ----------------------------------------------------------------------
#pragma unroll
    for (int l = 2; l < NLEV; ++l) {
      const int S = G >> (2 * (l - 1));
      const double* a = tree + Geo::lvl_off(l - 1);
      double* b = tree + Geo::lvl_off(l);
      for (int k = lane; k < S; k += 64) {
        double s = ((a[4 * k] + a[4 * k + 1]) + a[4 * k + 2]) + a[4 * k + 3];
        b[k] = s * 0.25;
      }
      __syncthreads();
    }

    // ---- index samples (core/streaming_index_builder.py:154-205) ------------------------------
    float rowv[(NS + 63) / 64];
    float rmin = __builtin_huge_valf(), rmax = -__builtin_huge_valf();
    const int lim = L > NS ? L : NS;
    for (int i = lane; i < lim; i += 64) {
      double val = 0.0;
      if (i < L) {
        int lev;
        int64_t pos;
        if (stream_sample(sched, i, lev, pos)) {
          if (lev == 0) val = (pos < d) ? (double)src[pos] : 0.0;
          else val = tree[Geo::lvl_off(lev) + pos];
        }
        if (idx_out) idx_out[e * (int64_t)L + i] = val;
      }
      if (i < NS) {
        float rv = (float)val;  // embed casts to the image dtype (core/index_generator.py:247)
        rowv[i / 64] = rv;
        rmin = fminf(rmin, rv);
        rmax = fmaxf(rmax, rv);
      }
    }
    mn = fminf(mn, wave_min(rmin));
    mx = fmaxf(mx, wave_max(rmax));

    // ---- quantize into the LDS frame ------------------------------------------------------------
    const bool flat = (mx == mn);
    const float rng = mx - mn;
    const uint32_t q0 = flat ? 128u : quant1(0.f, mn, rng);
    if (padded || flat) {
      const uint32_t w = q0 * 0x01010101u;
      uint4 w4 = make_uint4(w, w, w, w);
      for (int c = lane; c < NS * NS / 16; c += 64) reinterpret_cast<uint4*>(frame)[c] = w4;
      if (NS * NS < 16)
        for (int c = lane; c < NS * NS; c += 64) frame[c] = (uint8_t)q0;
      __syncthreads();
    }
    if (!flat) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int j = lane + 64 * t;
        if (j < groups_data && j < G) {
          float4 x;
          if constexpr (Geo::KEEP) {
            x = v[t];
          } else {
            x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (4 * j + 0 < d) x.x = src[4 * j + 0];
            if (4 * j + 1 < d) x.y = src[4 * j + 1];
            if (4 * j + 2 < d) x.z = src[4 * j + 2];
            if (4 * j + 3 < d) x.w = src[4 * j + 3];
          }
          const uint32_t q_0 = (4 * j + 0 < d) ? quant1(x.x, mn, rng) : q0;
          const uint32_t q_1 = (4 * j + 1 < d) ? quant1(x.y, mn, rng) : q0;
          const uint32_t q_2 = (4 * j + 2 < d) ? quant1(x.z, mn, rng) : q0;
          const uint32_t q_3 = (4 * j + 3 < d) ? quant1(x.w, mn, rng) : q0;
          const uint32_t ent = lut[j];
          const uint32_t code = ent >> 16;
          const uint32_t w = (q_0 << (8 * (code & 3))) | (q_1 << (8 * ((code >> 2) & 3))) |
                             (q_2 << (8 * ((code >> 4) & 3))) | (q_3 << (8 * ((code >> 6) & 3)));
          const uint32_t off = ent & 0xFFFFu;
          if constexpr (NS >= 2) {
            *reinterpret_cast<uint16_t*>(frame + off) = (uint16_t)(w & 0xFFFFu);
            *reinterpret_cast<uint16_t*>(frame + off + NS) = (uint16_t)(w >> 16);
          }
        }
      }
    }
    for (int i = lane; i < NS; i += 64) frame[NS * NS + i] = flat ? 128 : (uint8_t)quant1(rowv[i / 64], mn, rng);
    __syncthreads();

    // ---- stream the frame to HBM ---------------------------------------------------------------
    uint8_t* dst = frame_out + e * (int64_t)Geo::FB;
    if constexpr ((Geo::FB % 16) == 0) {
      for (int c = lane; c < Geo::FB / 16; c += 64)
        reinterpret_cast<uint4*>(dst)[c] = reinterpret_cast<const uint4*>(frame)[c];
    } else {
      for (int c = lane; c < Geo::FB; c += 64) dst[c] = frame[c];
    }
    if (minmax_out && lane == 0) {
      minmax_out[2 * e] = mn;
      minmax_out[2 * e + 1] = mx;
    }
    __syncthreads();
  }
}

template <int NS>
static int launch_fused(const float* in, int64_t N, int64_t stride, int d, int L, uint8_t* frame, double* idx,
                        float* minmax, hipStream_t s) {
  using Geo = FusedGeom<NS>;
  StreamSchedule sched;
  stream_schedule((int64_t)NS * NS, L, sched);
  const bool vec_ok = ((reinterpret_cast<uintptr_t>(in) & 15) == 0) && (stride % 4 == 0);
  size_t lds = Geo::lds_bytes();
  if (lds > 64 * 1024) HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_fused<NS>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if ((Geo::FB % 16) == 0 && (reinterpret_cast<uintptr_t>(frame) & 15) != 0)
    return fail(HQ_E_INVALID, "frame buffer must be 16-byte aligned");
  int grid = persistent_grid((const void*)k_fused<NS>, 64, lds, N);
  hipLaunchKernelGGL(k_fused<NS>, dim3(grid), dim3(64), lds, s, in, N, stride, d, L, vec_ok, sched, frame,
                     idx, minmax);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

// ------------------------------------------------------------------------------------------------
// standalone streaming index from an image (I1): gathers the Hilbert stream (map_from_2d) then the
// same tree + sampling.  One wave per image, tree in LDS (n <= 128).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(64) void k_stream_index(const T* __restrict__ img, int64_t N, uint32_t n, int L,
                                                     StreamSchedule sched, int tree_len,
                                                     double* __restrict__ out) {
  extern __shared__ double tr[];
  const int lane = threadIdx.x;
  const uint32_t G = sched.nlev > 1 ? (uint32_t)sched.size[1] : 0u;  // full groups of the stream
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const T* im = img + e * (int64_t)n * n;
    if (sched.nlev > 1) {
      for (uint32_t j = lane; j < G; j += 64) {
        double s = 0.0;
        for (uint32_t m = 0; m < 4; ++m) {
          uint32_t x, y;
          d2xy(n, 4 * j + m, x, y);
          double v = (double)im[y * n + x];
          s = (m == 0) ? v : s + v;
        }
        tr[j] = s * 0.25;
      }
    }
    __syncthreads();
    int off_prev = 0, off = (int)G;
    for (int l = 2; l < sched.nlev; ++l) {
      int S = (int)sched.size[l];
      for (int k = lane; k < S; k += 64) {
        const double* a = tr + off_prev + 4 * k;
        tr[off + k] = (((a[0] + a[1]) + a[2]) + a[3]) * 0.25;
      }
      __syncthreads();
      off_prev = off;
      off += S;
    }
    for (int i = lane; i < L; i += 64) {
      double val = 0.0;
      int lev;
      int64_t pos;
      if (stream_sample(sched, i, lev, pos)) {
        if (lev == 0) {
          uint32_t x, y;
          d2xy(n, (uint32_t)pos, x, y);
          val = (double)im[y * n + x];
        } else {
          int o = 0;
          for (int l = 1; l < lev; ++l) o += (int)sched.size[l];
          val = tr[o + pos];
        }
      }
      out[e * (int64_t)L + i] = val;
    }
    __syncthreads();
  }
  (void)tree_len;
}

// ------------------------------------------------------------------------------------------------
// Q1 standalone: per image min/max then quantize.  256 threads per image.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_quantize(const float* __restrict__ enh, int64_t N, int64_t cells,
                                                  uint8_t* __restrict__ out, float* __restrict__ minmax) {
  __shared__ float smin[4], smax[4];
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const float* p = enh + e * cells;
    float lmin = __builtin_huge_valf(), lmax = -__builtin_huge_valf();
    for (int64_t c = threadIdx.x; c < cells; c += 256) {
      float v = p[c];
      lmin = fminf(lmin, v);
      lmax = fmaxf(lmax, v);
    }
    lmin = wave_min(lmin);
    lmax = wave_max(lmax);
    if ((threadIdx.x & 63) == 0) { smin[threadIdx.x >> 6] = lmin; smax[threadIdx.x >> 6] = lmax; }
    __syncthreads();
    float mn = fminf(fminf(smin[0], smin[1]), fminf(smin[2], smin[3]));
    float mx = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    __syncthreads();
    const bool flat = mx == mn;
    const float rng = mx - mn;
    uint8_t* o = out + e * cells;
    for (int64_t c = threadIdx.x; c < cells; c += 256) o[c] = flat ? 128 : (uint8_t)quant1(p[c], mn, rng);
    if (minmax && threadIdx.x == 0) { minmax[2 * e] = mn; minmax[2 * e + 1] = mx; }
  }
}

// Q2: u8/255 * (mx - mn) + mn in float32 (core/compressor.py:301), constant -> mn (:297-298)
__global__ void k_dequantize(const uint8_t* __restrict__ u8, int64_t N, int64_t cells, const float* __restrict__ mm,
                             float* __restrict__ out) {
  int64_t total = N * cells;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t e = i / cells;
    float mn = mm[2 * e], mx = mm[2 * e + 1];
    float r;
    if (mx == mn) {
      r = mn;
    } else {
      float t = (float)u8[i] / 255.0f;
      t = t * (mx - mn);
      r = t + mn;
    }
    out[i] = r;
  }
}

}  // namespace hq

namespace hq {
int fused_fast(const float* in, int64_t N, int64_t stride, int d, int n, int L, uint8_t* frame, double* idx,
               float* mm, hipStream_t s);  // hq_fused.hip
}

using namespace hq;

extern "C" {

int hq_map_index_quantize(const float* in, int64_t N, int64_t in_stride, int d, int n, int L,
                          uint8_t* frame, double* idx, float* minmax, hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Dimension must be a power of 2, got %d", n);
  if (n < 2 || n > 128) return fail(HQ_E_UNSUPPORTED, "fused kernel supports 2 <= n <= 128, got %d", n);
  if (d < 0 || L < 0 || N < 0 || in_stride < d)
    return fail(HQ_E_INVALID, "bad shape N=%lld d=%d L=%d stride=%lld", (long long)N, d, L, (long long)in_stride);
  if ((int64_t)d > (int64_t)n * n)
    return fail(HQ_E_TOO_MANY, "Too many parameters (%d) for dimensions %dx%d (%d cells)", d, n, n, n * n);
  if (N == 0) return HQ_OK;
  if (!frame || (d > 0 && !in)) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (!opt_on(OPT_FUSED_GENERIC)) {  // software-pipelined path for n in {16, 32, 64}, L <= 64
    const int rc = fused_fast(in, N, in_stride, d, n, L, frame, idx, minmax, s);
    if (rc != HQ_E_UNSUPPORTED) return rc;
  }
  switch (n) {
    case 2: return launch_fused<2>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 4: return launch_fused<4>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 8: return launch_fused<8>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 16: return launch_fused<16>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 32: return launch_fused<32>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 64: return launch_fused<64>(in, N, in_stride, d, L, frame, idx, minmax, s);
    case 128: return launch_fused<128>(in, N, in_stride, d, L, frame, idx, minmax, s);
  }
  return fail(HQ_E_UNSUPPORTED, "n=%d", n);
}

int hq_index_streaming(int dtype, const void* img, int64_t N, int n, int stream_len, int L, double* idx_out,
                       hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Image must be square with power-of-2 dimensions, got %dx%d", n, n);
  if (n > 128) return fail(HQ_E_UNSUPPORTED, "streaming index supports n <= 128, got %d", n);
  if (L < 0 || N < 0 || stream_len < 0 || stream_len > n * n) return fail(HQ_E_INVALID, "bad shape");
  if (N == 0 || L == 0) return HQ_OK;
  if (!img || !idx_out) return fail(HQ_E_INVALID, "null buffer");
  StreamSchedule sched;
  stream_schedule((int64_t)stream_len, L, sched);
  int tree_len = 0;
  for (int l = 1; l < sched.nlev; ++l) tree_len += (int)sched.size[l];
  size_t lds = (size_t)(tree_len > 0 ? tree_len : 1) * 8;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == HQ_F32) {
    if (lds > 64 * 1024)
      HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_stream_index<float>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = persistent_grid((const void*)k_stream_index<float>, 64, lds, N);
    hipLaunchKernelGGL(k_stream_index<float>, dim3(grid), dim3(64), lds, s, (const float*)img, N, (uint32_t)n, L,
                       sched, tree_len, idx_out);
  } else if (dtype == HQ_F64) {
    if (lds > 64 * 1024)
      HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_stream_index<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = persistent_grid((const void*)k_stream_index<double>, 64, lds, N);
    hipLaunchKernelGGL(k_stream_index<double>, dim3(grid), dim3(64), lds, s, (const double*)img, N, (uint32_t)n, L,
                       sched, tree_len, idx_out);
  } else {
    return fail(HQ_E_UNSUPPORTED, "streaming index dtype %d (f32/f64 only)", dtype);
  }
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_quantize_u8(const float* enh, int64_t N, int rows, int cols, uint8_t* out, float* minmax, hq_stream_t stream) {
  if (N < 0 || rows < 0 || cols < 0) return fail(HQ_E_INVALID, "bad shape");
  int64_t cells = (int64_t)rows * cols;
  if (N == 0 || cells == 0) return HQ_OK;
  if (!enh || !out) return fail(HQ_E_INVALID, "null buffer");
  int grid = persistent_grid((const void*)k_quantize, 256, 0, N);
  hipLaunchKernelGGL(k_quantize, dim3(grid), dim3(256), 0, (hipStream_t)stream, enh, N, cells, out, minmax);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_dequantize_u8(const uint8_t* u8, int64_t N, int rows, int cols, const float* minmax, float* out,
                     hq_stream_t stream) {
  if (N < 0 || rows < 0 || cols < 0) return fail(HQ_E_INVALID, "bad shape");
  int64_t total = N * (int64_t)rows * cols;
  if (total == 0) return HQ_OK;
  if (!u8 || !out || !minmax) return fail(HQ_E_INVALID, "null buffer");
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_dequantize, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, u8, N,
                     (int64_t)rows * cols, minmax, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // extern "C"
