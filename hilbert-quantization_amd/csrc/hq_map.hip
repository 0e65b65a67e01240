// hq_map.hip — Hilbert coordinate tables and the 1-D <-> 2-D maps.
//
// Reference: core/hilbert_mapper.py:17-205 (and its RAG twin rag/embedding_generation/
// hilbert_mapper.py:16-204).  The reference rebuilds an n*n coordinate list in Python on every
// call and scatters element by element; here every output element is produced by one lane with
// the curve index computed from an LDS look-up table that the workgroup builds once, so HBM sees
// exactly one coalesced write of the image and one read of the input rows.
#include "hq_common.h"

#include <stdlib.h>
#include <string.h>

namespace hq {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// kernel-variant options: name table (hq_set_option), values set explicitly; DIAG builds also read
// HQ_<NAME> once at load
static const char* const kOptNames[OPT_COUNT] = {
    "fused_v", "fused_generic",
    "chunk_nt", "chunk_exactdiv", "chunk_generic", "chunk_wpb", "chunk_cpw",
    "precomp_nt", "precomp_tree_lds", "precomp_pad", "precomp_skip", "precomp_grid", "precomp_pf",
    "precomp_diag",
    "cos_kernel",
    "sample_stride", "sample_waves", "sample_kth", "sample_variant",
    "scan_v1", "scan_nosample", "scan_expt", "scan_variant", "scan_wpb", "scan_pf", "scan_nb", "ov_waves", "ov_occ",
    "refine_global", "refine_expt", "seg_prepare_flat", "select_2stage", "level_scores_v1", "scan_split3", "scan_occ", "scanov_split3", "sample_hi",
    "precomp_ws", "precomp_leaf_rot", "precomp_order", "scanov_v1", "ov_pf", "precomp_g2reg",
    "refine_coop", "precomp_compact", "prep_coop", "pool_sort_mem", "refine_small", "final_rounds",
    "rank_ct", "rank_win", "rank_sort_nt", "rank_sort_small"};
static int64_t g_opt_val[OPT_COUNT];
static bool g_opt_set[OPT_COUNT];

static int opt_find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < OPT_COUNT; ++i)
    if (strcmp(kOptNames[i], name) == 0) return i;
  return -1;
}

#ifdef HQ_DIAG
// diagnostics builds: HQ_FUSED_V=... etc. from the environment, read once when the library loads
__attribute__((constructor)) static void opt_from_env() {
  for (int i = 0; i < OPT_COUNT; ++i) {
    char env[64] = "HQ_";
    for (int k = 0; kOptNames[i][k] && k < 56; ++k) {
      const char c = kOptNames[i][k];
      env[3 + k] = (c >= 'a' && c <= 'z') ? (char)(c - 32) : c;
      env[4 + k] = 0;
    }
    const char* v = getenv(env);
    if (!v) continue;
    int64_t x = atoll(v);
    if (i == OPT_COS_KERNEL) x = strcmp(v, "regstage") == 0 ? 1 : strcmp(v, "lockstep") == 0 ? 2
                                 : strcmp(v, "temporal") == 0 ? 3 : x;
    g_opt_val[i] = x;
    g_opt_set[i] = true;
  }
}
#endif

int64_t opt(Opt id, int64_t dflt) { return g_opt_set[id] ? g_opt_val[id] : dflt; }

int persistent_grid(const void* kernel, int block, size_t dyn_lds, int64_t work_items) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, dyn_lds) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  int64_t g = (int64_t)cus * per_cu;
  if (g > work_items) g = work_items;
  if (g < 1) g = 1;
  return (int)g;
}

// ------------------------------------------------------------------------------------------------
// coordinate tables
// ------------------------------------------------------------------------------------------------
__global__ void k_table(uint32_t n, int32_t* xs, int32_t* ys, int32_t* tab_xy2d) {
  uint32_t total = n * n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    uint32_t x, y;
    d2xy(n, i, x, y);
    if (xs) xs[i] = (int32_t)x;
    if (ys) ys[i] = (int32_t)y;
    if (tab_xy2d) {
      // row-major cell i = (y*n + x) -> curve index, computed independently via xy2d
      uint32_t cx = i % n, cy = i / n;
      tab_xy2d[i] = (int32_t)xy2d(n, cx, cy);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// map_to_2d: out[e][y][x] = in[e][xy2d(x,y)] (or 0 beyond d).  T = element bit-container type.
// LUT of xy2d (u16) in LDS when n <= 128, computed on the fly otherwise.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_map_to_2d(const T* __restrict__ in, int64_t N, int64_t stride,
                                                   int d, uint32_t n, T* __restrict__ out) {
  extern __shared__ uint16_t lut[];
  const uint32_t cells = n * n;
  const bool use_lut = n <= 128;
  if (use_lut) {
    for (uint32_t c = threadIdx.x; c < cells; c += blockDim.x) lut[c] = (uint16_t)xy2d(n, c % n, c / n);
    __syncthreads();
  }
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const T* src = in + e * stride;
    T* dst = out + e * (int64_t)cells;
    for (uint32_t c = threadIdx.x; c < cells; c += blockDim.x) {
      uint32_t i = use_lut ? (uint32_t)lut[c] : xy2d(n, c % n, c / n);
      dst[c] = (i < (uint32_t)d) ? src[i] : T(0);
    }
  }
}

// map_from_2d: out[e][i] = img[e][y_i][x_i], i < d_out.  LUT of d2xy packed (x | y << 16).
template <typename T>
__global__ __launch_bounds__(256) void k_map_from_2d(const T* __restrict__ img, int64_t N, uint32_t n,
                                                     int d_out, T* __restrict__ out) {
  extern __shared__ uint32_t lut32[];
  const uint32_t cells = n * n;
  const bool use_lut = n <= 128;
  if (use_lut) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)d_out; i += blockDim.x) {
      uint32_t x, y;
      d2xy(n, i, x, y);
      lut32[i] = y * n + x;
    }
    __syncthreads();
  }
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const T* src = img + e * (int64_t)cells;
    T* dst = out + e * (int64_t)d_out;
    for (uint32_t i = threadIdx.x; i < (uint32_t)d_out; i += blockDim.x) {
      uint32_t off;
      if (use_lut) {
        off = lut32[i];
      } else {
        uint32_t x, y;
        d2xy(n, i, x, y);
        off = y * n + x;
      }
      dst[i] = src[off];
    }
  }
}

template <typename T>
static int launch_map_to_2d(const void* in, int64_t N, int64_t stride, int d, int n, void* out,
                            hipStream_t s) {
  size_t lds = (n <= 128) ? (size_t)n * n * sizeof(uint16_t) : 0;
  int grid = persistent_grid((const void*)k_map_to_2d<T>, 256, lds, N);
  hipLaunchKernelGGL(k_map_to_2d<T>, dim3(grid), dim3(256), lds, s, (const T*)in, N, stride, d,
                     (uint32_t)n, (T*)out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <typename T>
static int launch_map_from_2d(const void* img, int64_t N, int n, int d_out, void* out, hipStream_t s) {
  size_t lds = (n <= 128) ? (size_t)d_out * sizeof(uint32_t) : 0;
  int grid = persistent_grid((const void*)k_map_from_2d<T>, 256, lds, N);
  hipLaunchKernelGGL(k_map_from_2d<T>, dim3(grid), dim3(256), lds, s, (const T*)img, N, (uint32_t)n,
                     d_out, (T*)out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_version(void) { return 1; }

const char* hq_last_error(void) { return g_err; }

int hq_set_option(const char* name, int64_t value) {
  const int i = opt_find(name);
  if (i < 0) return fail(HQ_E_INVALID, "unknown option '%s'", name ? name : "(null)");
  g_opt_val[i] = value;
  g_opt_set[i] = true;
  return HQ_OK;
}

int hq_reset_option(const char* name) {
  const int i = opt_find(name);
  if (i < 0) return fail(HQ_E_INVALID, "unknown option '%s'", name ? name : "(null)");
  g_opt_set[i] = false;
  return HQ_OK;
}

int hq_get_option(const char* name, int64_t* value) {
  const int i = opt_find(name);
  if (i < 0) return fail(HQ_E_INVALID, "unknown option '%s'", name ? name : "(null)");
  if (value) *value = g_opt_val[i];
  return g_opt_set[i] ? 1 : 0;
}

int hq_diag_build(void) {
#ifdef HQ_DIAG
  return 1;
#else
  return 0;
#endif
}

int hq_hilbert_table(int n, int32_t* xs, int32_t* ys, int32_t* tab, hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Grid size must be a power of 2, got %d", n);
  if ((int64_t)n * n > (int64_t)1 << 30) return fail(HQ_E_INVALID, "grid too large: %d", n);
  int64_t total = (int64_t)n * n;
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_table, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint32_t)n, xs, ys, tab);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_map_to_2d(int dtype, const void* in, int64_t N, int64_t in_stride, int d, int n, void* out,
                 hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Dimension must be a power of 2, got %d", n);
  if (d < 0 || N < 0 || in_stride < d) return fail(HQ_E_INVALID, "bad shape N=%lld d=%d stride=%lld",
                                                   (long long)N, d, (long long)in_stride);
  if ((int64_t)d > (int64_t)n * n)
    return fail(HQ_E_TOO_MANY, "Too many parameters (%d) for dimensions %dx%d (%lld cells)", d, n, n,
                (long long)n * n);
  if (N == 0) return HQ_OK;
  if (!out || (d > 0 && !in)) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  switch (dtype_size(dtype)) {
    case 1: return launch_map_to_2d<uint8_t>(in, N, in_stride, d, n, out, s);
    case 2: return launch_map_to_2d<uint16_t>(in, N, in_stride, d, n, out, s);
    case 4: return launch_map_to_2d<uint32_t>(in, N, in_stride, d, n, out, s);
    case 8: return launch_map_to_2d<uint64_t>(in, N, in_stride, d, n, out, s);
    default: return fail(HQ_E_INVALID, "unknown dtype code %d", dtype);
  }
}

int hq_map_from_2d(int dtype, const void* img, int64_t N, int n, int d_out, void* out,
                   hq_stream_t stream) {
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Dimension must be a power of 2, got %d", n);
  if (d_out < 0 || (int64_t)d_out > (int64_t)n * n || N < 0)
    return fail(HQ_E_INVALID, "bad shape N=%lld n=%d d_out=%d", (long long)N, n, d_out);
  if (N == 0 || d_out == 0) return HQ_OK;
  if (!img || !out) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  switch (dtype_size(dtype)) {
    case 1: return launch_map_from_2d<uint8_t>(img, N, n, d_out, out, s);
    case 2: return launch_map_from_2d<uint16_t>(img, N, n, d_out, out, s);
    case 4: return launch_map_from_2d<uint32_t>(img, N, n, d_out, out, s);
    case 8: return launch_map_from_2d<uint64_t>(img, N, n, d_out, out, s);
    default: return fail(HQ_E_INVALID, "unknown dtype code %d", dtype);
  }
}

int hq_parse_structure(int L, int32_t* out, int max_levels) {
  SegTable t;
  parse_structure(L, L, t);
  int k = t.nseg < max_levels ? t.nseg : max_levels;
  for (int i = 0; i < k && out; ++i) {
    out[4 * i + 0] = t.grid[i];
    out[4 * i + 1] = t.start[i];
    out[4 * i + 2] = t.end[i];
    out[4 * i + 3] = t.offset[i];
  }
  return t.nseg;
}

}  // extern "C"
