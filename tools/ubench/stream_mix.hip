// Microbenchmark: HBM rate of the fused kernel's traffic shape (6144 B read + W B written per item,
// one wave per item, persistent grid) against a plain float4 copy.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f4v __attribute__((ext_vector_type(4)));
template <int MODE>  // 0 plain, 1 nt store, 2 nt load + nt store
__global__ __launch_bounds__(64) void k_copy(const float4* __restrict__ in, float4* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * 64 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 64) {
    if (MODE == 0) out[i] = in[i];
    else {
      f4v v = MODE == 2 ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(in) + i) : reinterpret_cast<const f4v*>(in)[i];
      __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(out) + i);
    }
  }
}
// read-only: sum, one store per thread
__global__ __launch_bounds__(64) void k_read(const float4* __restrict__ in, float* __restrict__ out, int64_t n) {
  float s = 0.f;
  for (int64_t i = blockIdx.x * 64 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 64) { const float4 v = in[i]; s += v.x + v.y + v.z + v.w; }
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// item e: read 384 float4 (6144 B), write W bytes (uint4 per lane), 2-deep prefetch
template <int W, bool RUN>
__global__ __launch_bounds__(64) void k_items(const float4* __restrict__ in, uint8_t* __restrict__ out, int64_t N,
                                              int64_t run) {
  const int lane = threadIdx.x;
  int64_t e0, e1, step;
  if (RUN) { e0 = blockIdx.x * run; e1 = e0 + run; if (e1 > N) e1 = N; step = 1; }
  else { e0 = blockIdx.x; e1 = N; step = gridDim.x; }
  float4 a[6], b[6];
  auto ld = [&](int64_t e, float4* d) {
#pragma unroll
    for (int t = 0; t < 6; ++t) d[t] = in[e * 384 + lane + 64 * t];
  };
  if (e0 < e1) ld(e0, a);
  for (int64_t e = e0; e < e1; e += step) {
    if (e + step < e1) ld(e + step, b);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 6; ++t) s += a[t].x + a[t].y + a[t].z + a[t].w;
    const uint32_t v = __float_as_uint(s);
    uint8_t* dst = out + e * W;
    for (int c = lane; c < W / 16; c += 64) reinterpret_cast<uint4*>(dst)[c] = make_uint4(v, v, v, v);
#pragma unroll
    for (int t = 0; t < 6; ++t) a[t] = b[t];
  }
}

template <int W, bool RUN>
void run_items(const float4* in, uint8_t* out, int64_t N, int grid, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int64_t run = (N + grid - 1) / grid;
  hipLaunchKernelGGL((k_items<W, RUN>), dim3(grid), dim3(64), 0, 0, in, out, N, run);
  (void)hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_items<W, RUN>), dim3(grid), dim3(64), 0, 0, in, out, N, run);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  printf("%-28s grid %6d: %.3f ms, %.2f TB/s (read+write)\n", name, grid, ms, (double)N * (6144 + W) / (ms * 1e-3) / 1e12);
}

int main() {
  const int64_t N = 1000000;
  float4* in;
  uint8_t* out;
  (void)hipMalloc(&in, N * 6144);
  (void)hipMalloc(&out, N * 6144);
  (void)hipMemset(in, 0, N * 6144);
  {
    const int64_t n = N * 6144 / 16 / 2;  // copy 3 GB -> 3 GB
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 4; ++mode) {
      for (int grid : {16384, 65536}) {
        auto launch = [&]() {
          if (mode == 0) hipLaunchKernelGGL(k_copy<0>, dim3(grid), dim3(64), 0, 0, in, (float4*)out, n);
          if (mode == 1) hipLaunchKernelGGL(k_copy<1>, dim3(grid), dim3(64), 0, 0, in, (float4*)out, n);
          if (mode == 2) hipLaunchKernelGGL(k_copy<2>, dim3(grid), dim3(64), 0, 0, in, (float4*)out, n);
          if (mode == 3) hipLaunchKernelGGL(k_read, dim3(grid), dim3(64), 0, 0, in, (float*)out, 2 * n);
        };
        launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < 5; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        printf("%s grid %d: %.3f ms, %.2f TB/s\n", mode == 0 ? "copy plain" : mode == 1 ? "copy nt-store" : mode == 2 ? "copy nt-both" : "read only",
               grid, ms, 2.0 * n * 16 / (ms * 1e-3) / 1e12);
      }
    }
  }
  for (int g : {3072, 4096, 8192, 16384}) {
    run_items<4160, false>(in, out, N, g, "items W=4160 strided");
    run_items<4160, true>(in, out, N, g, "items W=4160 runs");
    run_items<4096, false>(in, out, N, g, "items W=4096 strided");

  }
  return 0;
}
