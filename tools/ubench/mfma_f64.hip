// Microbenchmark: v_mfma_f64_16x16x4f64 throughput on gfx950 vs number of independent
// accumulation chains, waves per SIMD, and interleaved f64 VALU work.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int CH, int VALU>
__global__ __launch_bounds__(64) void k(double* out, int iters, double x) {
  dbl4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = dbl4{0, 0, 0, 0};
  double a = x + threadIdx.x, b = x * 2.0 + threadIdx.x;
  double v0 = a, v1 = b, v2 = a * b, v3 = a + b;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
#pragma unroll
      for (int u = 0; u < VALU; ++u) {
        v0 = fma(v0, v1, v2);
        v1 = fma(v1, v2, v3);
        v2 = fma(v2, v3, v0);
        v3 = fma(v3, v0, v1);
      }
    }
  }
  double s = v0 + v1 + v2 + v3;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// f64 VALU FMA only: 8 independent chains per lane
__global__ __launch_bounds__(64) void kv(double* out, int iters, double x) {
  double v[8];
  for (int c = 0; c < 8; ++c) v[c] = x + threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = fma(v[c], 0.999, 0.001);
  }
  double s = 0;
  for (int c = 0; c < 8; ++c) s += v[c];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

void runv(int waves_per_simd, double* out) {
  const int blocks = 256 * 4 * waves_per_simd;
  const int iters = 4000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kv, dim3(blocks), dim3(64), 0, 0, out, iters, 1.0);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kv, dim3(blocks), dim3(64), 0, 0, out, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double fmas = (double)blocks * 64 * iters * 32;
  printf("VALU f64 fma waves/simd=%d : %.3f ms, %.1f TF\n", waves_per_simd, ms, fmas * 2 / (ms * 1e-3) / 1e12);
}

template <int CH, int VALU>
void run(int waves_per_simd, double* out) {
  const int blocks = 256 * 4 * waves_per_simd;
  const int iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k<CH, VALU>), dim3(blocks), dim3(64), 0, 0, out, iters, 1.0);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<CH, VALU>), dim3(blocks), dim3(64), 0, 0, out, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfma = (double)blocks * iters * CH;
  const double per_simd = mfma / 1024.0;
  const double cyc = ms * 1e-3 * 2.4e9 / per_simd;
  printf("chains=%d valu4x%d waves/simd=%d : %.3f ms, %.1f cycles/MFMA/SIMD @2.4GHz, %.1f TF\n", CH, VALU,
         waves_per_simd, ms, cyc, mfma * 2048 / (ms * 1e-3) / 1e12);
}

int main() {
  double* out;
  (void)hipMalloc(&out, 256 * 4 * 8 * 64 * 8);
  for (int w = 1; w <= 8; w *= 2) runv(w, out);
  for (int w = 4; w <= 8; w *= 2) {
    run<4, 0>(w, out);
    run<8, 0>(w, out);
    run<4, 2>(w, out);
  }
  for (int w = 1; w <= 2; ++w) {
    run<1, 0>(w, out);
    run<2, 0>(w, out);
    run<4, 0>(w, out);
    run<8, 0>(w, out);
    run<4, 1>(w, out);
    run<4, 2>(w, out);
    run<4, 4>(w, out);
    run<8, 2>(w, out);
  }
  return 0;
}
