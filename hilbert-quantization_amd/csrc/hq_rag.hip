// hq_rag.hip — the RAG engine's remaining scoring pieces:
//   * cosine of float32 OR float64 rows (rag/search/engine.py:622-660): float64 inputs stay float64
//     (the reference computes np.dot / np.linalg.norm in the input dtype);
//   * _detect_original_embedding_height / _extract_original_embedding (engine.py:134-162, 604-620) and
//     _calculate_spatial_locality_similarity (engine.py:662-714) for Q query x N stored enhanced images;
//   * _apply_progressive_threshold (engine.py:243-287) as an order-preserving device select.
// Dot products and norms accumulate in float64 (the reference's BLAS sdot/ddot/nrm2 orders are not
// reproducible; |err| < 1e-12 relative for f64 inputs, < 1e-6 against the reference's float32 values).
// Window means follow NumPy's pairwise order over the reference's list of window scores.
#include "hq_common.h"

#include <math.h>

namespace hq {

template <typename T>
__global__ __launch_bounds__(256) void k_cosine_t(const T* __restrict__ A, int Q, const T* __restrict__ B, int64_t N,
                                                  int K, double* __restrict__ out) {
  const int64_t total = (int64_t)Q * N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const T* a = A + (t / N) * K;
    const T* b = B + (t % N) * K;
    double dot = 0.0, na = 0.0, nb = 0.0;
    for (int i = 0; i < K; ++i) {
      const double x = (double)a[i], y = (double)b[i];
      dot = fma(x, y, dot);
      na = fma(x, x, na);
      nb = fma(y, y, nb);
    }
    out[t] = (na != 0.0 && nb != 0.0) ? (dot / (sqrt(na) * sqrt(nb)) + 1.0) / 2.0 : 0.0;
  }
}

// _detect_original_embedding_height (engine.py:134-162): from the bottom row up, the first row whose zero
// ratio np.sum(row == 0) / W is below 0.5 ends the original embedding (height = row + 1); H if none.
// zeros / W < 0.5 <=> 2 zeros < W exactly (W < 2^24: the quotient is never within an ulp of 0.5).
// Block-cooperative: every thread takes rows, the largest qualifying row wins (LDS atomicMax).
template <typename T>
__device__ int detect_height(const T* img, int H, int W, int* slot) {
  if (threadIdx.x == 0) *slot = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < H; r += blockDim.x) {
    int z = 0;
    for (int c = 0; c < W; ++c) z += img[(int64_t)r * W + c] == (T)0 ? 1 : 0;
    if (2 * z < W) atomicMax(slot, r + 1);
  }
  __syncthreads();
  const int h = *slot;
  __syncthreads();
  return h > 0 ? h : H;
}

template <typename T>
__global__ __launch_bounds__(64) void k_detect_heights(const T* __restrict__ imgs, int64_t N, int H, int W,
                                                       int* __restrict__ out) {
  __shared__ int slot;
  for (int64_t i = blockIdx.x; i < N; i += gridDim.x) {
    const int h = detect_height(imgs + i * (int64_t)H * W, H, W, &slot);
    if (threadIdx.x == 0) out[i] = h;
  }
}

// (cos + 1) / 2 of two ws x ws windows (or of two whole h x W blocks, ws = 0) of row-major images
template <typename T>
__device__ __forceinline__ double window_cos(const T* a, const T* b, int W, int rows, int cols) {
  double dot = 0.0, na = 0.0, nb = 0.0;
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
      const double x = (double)a[(int64_t)r * W + c], y = (double)b[(int64_t)r * W + c];
      dot = fma(x, y, dot);
      na = fma(x, x, na);
      nb = fma(y, y, nb);
    }
  return (na != 0.0 && nb != 0.0) ? (dot / (sqrt(na) * sqrt(nb)) + 1.0) / 2.0 : 0.0;
}

// _calculate_spatial_locality_similarity (engine.py:662-714) for every (query, stored image) pair: one
// 256-thread workgroup per pair.  Both images' original heights are detected (the index rows appended
// by the RAG generator are cut off, engine.py:604-620); different heights -> 0.0; window side
// ws = min(4, h // 4, W // 4); ws < 2 -> one cosine over the h x W block; else windows at stride ws / 2
// in (row, column) order, their scores kept in LDS and averaged in NumPy's pairwise order (np.mean of
// the reference's list).
template <typename T>
__global__ __launch_bounds__(256) void k_spatial(const T* __restrict__ Qi, int Qn, const T* __restrict__ Ci, int64_t N,
                                                 int H, int W, double* __restrict__ out) {
  extern __shared__ double wv[];
  __shared__ int slot;
  const int64_t img = (int64_t)H * W;
  for (int64_t t = blockIdx.x; t < (int64_t)Qn * N; t += gridDim.x) {
    const T* a = Qi + (t / N) * img;
    const T* b = Ci + (t % N) * img;
    const int ha = detect_height(a, H, W, &slot);
    const int hb = detect_height(b, H, W, &slot);
    double res = 0.0;
    if (ha == hb) {
      const int h = ha;
      int ws = 4;
      if (h / 4 < ws) ws = h / 4;
      if (W / 4 < ws) ws = W / 4;
      if (ws < 2) {
        if (threadIdx.x == 0) res = window_cos(a, b, W, h, W);
      } else {
        const int st = ws / 2;
        const int ni = (h - ws) / st + 1, nj = (W - ws) / st + 1;
        const int nw = ni * nj;
        for (int w = threadIdx.x; w < nw; w += blockDim.x) {
          const int i = (w / nj) * st, j = (w % nj) * st;
          wv[w] = window_cos(a + (int64_t)i * W + j, b + (int64_t)i * W + j, W, ws, ws);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          auto f = [&](int k) -> double { return wv[k]; };
          res = np_sum<double>(f, nw) / (double)nw;
        }
      }
    }
    if (threadIdx.x == 0) out[t] = res;
    __syncthreads();
  }
}

// _apply_progressive_threshold (engine.py:243-287) per row, order preserving: the first `cap` entries
// (in the caller's candidate order) whose score is >= thr.  One wave per row, 64 entries per ballot.
__global__ __launch_bounds__(64) void k_threshold_select(const double* __restrict__ sc, const int64_t* __restrict__ ids,
                                                         int Q, int64_t N, double thr, int64_t cap,
                                                         int64_t* __restrict__ out_ids, int64_t* __restrict__ out_n) {
  const int lane = threadIdx.x;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    int64_t n = 0;
    for (int64_t i0 = 0; i0 < N && n < cap; i0 += 64) {
      const int64_t i = i0 + lane;
      const bool ok = i < N && sc[(int64_t)q * N + i] >= thr;
      const unsigned long long m = __ballot(ok);
      const int64_t pos = n + __popcll(m & ((1ull << lane) - 1ull));
      if (ok && pos < cap) out_ids[(int64_t)q * cap + pos] = ids ? ids[(int64_t)q * N + i] : i;
      n += __popcll(m);
    }
    if (n > cap) n = cap;
    for (int64_t j = n + lane; j < cap; j += 64) out_ids[(int64_t)q * cap + j] = -1;
    if (lane == 0) out_n[q] = n;
  }
}

static int grid_for(int64_t work, int per) {
  int64_t g = (work + per - 1) / per;
  if (g > 65536) g = 65536;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_cosine_scores_dt(int dtype, const void* a, int Q, const void* b, int64_t N, int K, double* out,
                        hq_stream_t stream) {
  if (Q < 0 || N < 0 || K < 0) return fail(HQ_E_INVALID, "bad shape");
  if (dtype != HQ_F32 && dtype != HQ_F64) return fail(HQ_E_UNSUPPORTED, "dtype %d (float32 / float64)", dtype);
  if (Q == 0 || N == 0) return HQ_OK;
  if (!a || !b || !out) return fail(HQ_E_INVALID, "null buffer");
  const int g = grid_for((int64_t)Q * N, 256);
  if (dtype == HQ_F32)
    hipLaunchKernelGGL(k_cosine_t<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)a, Q,
                       (const float*)b, N, K, out);
  else
    hipLaunchKernelGGL(k_cosine_t<double>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const double*)a, Q,
                       (const double*)b, N, K, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_detect_heights(int dtype, const void* imgs, int64_t N, int H, int W, int* out, hq_stream_t stream) {
  if (N < 0 || H <= 0 || W <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (dtype != HQ_F32 && dtype != HQ_F64) return fail(HQ_E_UNSUPPORTED, "dtype %d (float32 / float64)", dtype);
  if (N == 0) return HQ_OK;
  if (!imgs || !out) return fail(HQ_E_INVALID, "null buffer");
  const int g = grid_for(N, 1);
  if (dtype == HQ_F32)
    hipLaunchKernelGGL(k_detect_heights<float>, dim3(g), dim3(64), 0, (hipStream_t)stream, (const float*)imgs, N, H,
                       W, out);
  else
    hipLaunchKernelGGL(k_detect_heights<double>, dim3(g), dim3(64), 0, (hipStream_t)stream, (const double*)imgs, N,
                       H, W, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_spatial_locality(int dtype, const void* q, int Q, const void* c, int64_t N, int H, int W, double* out,
                        hq_stream_t stream) {
  if (Q < 0 || N < 0 || H <= 0 || W <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (dtype != HQ_F32 && dtype != HQ_F64) return fail(HQ_E_UNSUPPORTED, "dtype %d (float32 / float64)", dtype);
  if (Q == 0 || N == 0) return HQ_OK;
  if (!q || !c || !out) return fail(HQ_E_INVALID, "null buffer");
  // window scores of one pair in LDS: at most ((H - 2) / 1 + 1) * ((W - 2) / 1 + 1) windows (ws = 2)
  const int64_t nw = (int64_t)(H / 1) * (W / 1);
  const size_t lds = (size_t)8 * (size_t)(nw < 8 ? 8 : nw);
  if (lds > 64 * 1024) return fail(HQ_E_UNSUPPORTED, "image %dx%d: window list exceeds 64 KiB of LDS", H, W);
  const int g = grid_for((int64_t)Q * N, 1);
  if (dtype == HQ_F32) {
    HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_spatial<float>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_spatial<float>, dim3(g), dim3(256), lds, (hipStream_t)stream, (const float*)q, Q,
                       (const float*)c, N, H, W, out);
  } else {
    HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_spatial<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_spatial<double>, dim3(g), dim3(256), lds, (hipStream_t)stream, (const double*)q, Q,
                       (const double*)c, N, H, W, out);
  }
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_threshold_select(const double* scores, const int64_t* ids, int Q, int64_t N, double threshold, int64_t cap,
                        int64_t* out_ids, int64_t* out_count, hq_stream_t stream) {
  if (Q < 0 || N < 0 || cap < 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || cap == 0) return HQ_OK;
  if ((N > 0 && !scores) || !out_ids || !out_count) return fail(HQ_E_INVALID, "null buffer");
  hipLaunchKernelGGL(k_threshold_select, dim3(Q < 8192 ? Q : 8192), dim3(64), 0, (hipStream_t)stream, scores, ids, Q,
                     N, threshold, cap, out_ids, out_count);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // extern "C"
