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

template <int NS>
static int launch_chunk(const uint16_t* in, int64_t total, int chunk, int64_t c0, int64_t c1, uint8_t* frame,
                        int64_t fstride, float* idx, int64_t istride, float* mm, hipStream_t s) {
  int L = NS;  // min(1024, n) (core/streaming_processor.py:897-899)
  TradPlan plan;
  trad_plan(NS, L, plan);
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
