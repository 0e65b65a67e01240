// Microbenchmark: which launch shape moves the fused kernel's traffic (6144 B read, 4160 B frame +
// 512 B index + 8 B min/max written per item) fastest on MI355X, next to tuned float4 copies.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_shapes hbm_shapes.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// copy with U float4 per thread in flight (all loads, then all stores), grid-stride
template <int U>
__global__ __launch_bounds__(256) void k_copyU(const float4* __restrict__ in, float4* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (b + 256 * u < n) ? in[b + 256 * u] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + 256 * u < n) out[b + 256 * u] = v[u];
  }
}
template <int U>
__global__ __launch_bounds__(256) void k_readU(const float4* __restrict__ in, float* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  float s = 0.f;
  for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + 256 * u < n) {
        const float4 v = in[b + 256 * u];
        s += (v.x + v.y) + (v.z + v.w);
      }
  }
  if (s == 1234.5f) out[0] = s;
}

// one item per wave, WPB waves per block, no loop (the hardware dispatcher is the scheduler)
template <int WPB, bool IDX>
__global__ __launch_bounds__(64 * WPB) void k_item1(const float4* __restrict__ in, uint8_t* __restrict__ fr,
                                                   double* __restrict__ idx, float* __restrict__ mm, int64_t N) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (e >= N) return;
  float4 a[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) a[t] = in[e * 384 + lane + 64 * t];
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 6; ++t) s += (a[t].x + a[t].y) + (a[t].z + a[t].w);
  const uint32_t v = __float_as_uint(s);
  uint4* dst = reinterpret_cast<uint4*>(fr + e * 4160);
  for (int c = lane; c < 260; c += 64) dst[c] = make_uint4(v, v, c, lane);
  if (IDX) {
    if ((lane & 1) == 0 && lane < 64) reinterpret_cast<double2*>(idx + e * 64)[lane >> 1] = make_double2(s, s);
    if (lane == 0) reinterpret_cast<float2*>(mm)[e] = make_float2(s, s);
  }
}

// persistent: WPB waves per block, each wave strides over items with PF items of prefetch
template <int WPB, int PF>
__global__ __launch_bounds__(64 * WPB) void k_itemP(const float4* __restrict__ in, uint8_t* __restrict__ fr,
                                                   double* __restrict__ idx, float* __restrict__ mm, int64_t N) {
  const int lane = threadIdx.x & 63;
  const int64_t G = (int64_t)gridDim.x * WPB;
  int64_t e = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  float4 a[PF + 1][6];
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (e + p * G < N)
#pragma unroll
      for (int t = 0; t < 6; ++t) a[p][t] = in[(e + p * G) * 384 + lane + 64 * t];
  for (; e < N; e += G) {
    if (e + PF * G < N)
#pragma unroll
      for (int t = 0; t < 6; ++t) a[PF][t] = in[(e + PF * G) * 384 + lane + 64 * t];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 6; ++t) s += (a[0][t].x + a[0][t].y) + (a[0][t].z + a[0][t].w);
    const uint32_t v = __float_as_uint(s);
    uint4* dst = reinterpret_cast<uint4*>(fr + e * 4160);
    for (int c = lane; c < 260; c += 64) dst[c] = make_uint4(v, v, c, lane);
    if ((lane & 1) == 0) reinterpret_cast<double2*>(idx + e * 64)[lane >> 1] = make_double2(s, s);
    if (lane == 0) reinterpret_cast<float2*>(mm)[e] = make_float2(s, s);
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int t = 0; t < 6; ++t) a[p][t] = a[p + 1][t];
  }
}

static hipEvent_t E0, E1;
template <class F>
static float time_it(F f, int reps = 10) {
  f();
  (void)hipEventRecord(E0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(E1);
  (void)hipEventSynchronize(E1);
  float ms;
  (void)hipEventElapsedTime(&ms, E0, E1);
  return ms / reps;
}

int main() {
  (void)hipEventCreate(&E0);
  (void)hipEventCreate(&E1);
  const int64_t N = 1000000;
  float4* in;
  uint8_t* fr;
  double* idx;
  float* mm;
  (void)hipMalloc(&in, N * 6144);
  (void)hipMalloc(&fr, N * 6144);
  (void)hipMalloc(&idx, N * 512);
  (void)hipMalloc(&mm, N * 8);
  (void)hipMemset(in, 1, N * 6144);
  const int64_t n4 = N * 6144 / 16 / 2;  // 3.07 GB -> 3.07 GB
  const double cbytes = 2.0 * n4 * 16;
#define COPY(U, GRID)                                                                                             \
  {                                                                                                               \
    const float ms = time_it([&] { hipLaunchKernelGGL(k_copyU<U>, dim3(GRID), dim3(256), 0, 0, in, (float4*)fr, n4); }); \
    printf("copy  U=%d grid=%7d : %.3f ms %.2f TB/s\n", U, GRID, ms, cbytes / ms / 1e9);                         \
  }
#define READ(U, GRID)                                                                                             \
  {                                                                                                               \
    const float ms = time_it([&] { hipLaunchKernelGGL(k_readU<U>, dim3(GRID), dim3(256), 0, 0, in, (float*)fr, 2 * n4); }); \
    printf("read  U=%d grid=%7d : %.3f ms %.2f TB/s\n", U, GRID, ms, cbytes / ms / 1e9);                         \
  }
  COPY(1, 4096) COPY(1, 16384) COPY(1, 65536) COPY(1, 750000)
  COPY(2, 4096) COPY(2, 16384) COPY(2, 65536)
  COPY(4, 2048) COPY(4, 4096) COPY(4, 16384)
  COPY(8, 1024) COPY(8, 2048) COPY(8, 4096)
  READ(1, 65536) READ(4, 4096) READ(4, 16384) READ(8, 2048) READ(8, 4096)
  const double ib = (double)N * (6144 + 4160 + 512 + 8);
#define ITEM1(WPB, IDX)                                                                                            \
  {                                                                                                                \
    const int g = (int)((N + WPB - 1) / WPB);                                                                      \
    const float ms = time_it([&] { hipLaunchKernelGGL((k_item1<WPB, IDX>), dim3(g), dim3(64 * WPB), 0, 0, in, fr, idx, mm, N); }); \
    printf("item1 WPB=%d idx=%d       : %.3f ms %.2f TB/s (%.0fM items/s)\n", WPB, IDX, ms, ib / ms / 1e9, N / ms / 1e3); \
  }
  ITEM1(1, true) ITEM1(2, true) ITEM1(4, true) ITEM1(8, true) ITEM1(4, false)
#define ITEMP(WPB, PF, GRID)                                                                                       \
  {                                                                                                                \
    const float ms = time_it([&] { hipLaunchKernelGGL((k_itemP<WPB, PF>), dim3(GRID), dim3(64 * WPB), 0, 0, in, fr, idx, mm, N); }); \
    printf("itemP WPB=%d PF=%d grid=%6d: %.3f ms %.2f TB/s (%.0fM items/s)\n", WPB, PF, GRID, ms, ib / ms / 1e9, N / ms / 1e3); \
  }
  ITEMP(1, 1, 2048) ITEMP(1, 1, 4096) ITEMP(1, 2, 2048) ITEMP(1, 2, 3584) ITEMP(1, 2, 4096)
  ITEMP(4, 1, 1024) ITEMP(4, 2, 512) ITEMP(4, 2, 896) ITEMP(4, 2, 1024) ITEMP(2, 2, 1792)
  return 0;
}
