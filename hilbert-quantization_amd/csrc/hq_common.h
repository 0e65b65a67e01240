// hq_common.h — shared device/host helpers for libhq_mi355x (gfx950 only).
//
// Integer Hilbert maths follows the reference's core/hilbert_mapper.py:42-113 (d2xy, xy2d, rotate);
// the streaming-index sample schedule follows core/streaming_index_builder.py:154-243 and the level
// structure parser core/search_engine.py:42-109.  Arithmetic that must be bit-exact (f32 IEEE
// division, f64 left-to-right sums) is compiled with -ffp-contract=off and without fast-math.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/hq_mi355x.h"

namespace hq {

// ------------------------------------------------------------------------------------------------
// error plumbing: thread-local last error, negative HQ_E_* codes (C-ABI contract, include/hq_mi355x.h)
// ------------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define HQ_CHECK_HIP(expr)                                                                   \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return ::hq::fail(HQ_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));            \
  } while (0)

#define HQ_CHECK_LAUNCH()                                                                    \
  do {                                                                                       \
    hipError_t _e = hipGetLastError();                                                       \
    if (_e != hipSuccess) return ::hq::fail(HQ_E_HIP, "kernel launch: %s", hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------------------------------------
// kernel-variant options (hq_set_option, include/hq_mi355x.h).  The library never reads the
// environment in a default build: a variant is selected only by an explicit hq_set_option call
// (parity tests, A/B tools).  `make DIAG=1` builds also take HQ_<NAME> from the environment once, at
// load.  opt(id, dflt) = the set value, else the call site's default.
// ------------------------------------------------------------------------------------------------
enum Opt {
  OPT_FUSED_V, OPT_FUSED_GENERIC,
  OPT_CHUNK_NT, OPT_CHUNK_EXACTDIV, OPT_CHUNK_GENERIC, OPT_CHUNK_WPB, OPT_CHUNK_CPW,
  OPT_PRECOMP_NT, OPT_PRECOMP_TREE_LDS, OPT_PRECOMP_PAD, OPT_PRECOMP_SKIP, OPT_PRECOMP_GRID, OPT_PRECOMP_PF,
  OPT_PRECOMP_DIAG,
  OPT_COS_KERNEL,
  OPT_SAMPLE_STRIDE, OPT_SAMPLE_WAVES, OPT_SAMPLE_KTH, OPT_SAMPLE_VARIANT,
  OPT_SCAN_V1, OPT_SCAN_NOSAMPLE, OPT_SCAN_EXPT, OPT_SCAN_VARIANT, OPT_SCAN_WPB, OPT_SCAN_PF, OPT_SCAN_NB, OPT_OV_WAVES, OPT_OV_OCC,
  OPT_REFINE_GLOBAL, OPT_REFINE_EXPT, OPT_SEG_PREPARE_FLAT, OPT_SELECT_2STAGE, OPT_LEVEL_SCORES_V1, OPT_SCAN_SPLIT3, OPT_SCAN_OCC, OPT_SCANOV_SPLIT3, OPT_SAMPLE_HI,
  OPT_PRECOMP_WS, OPT_PRECOMP_LEAF_ROT, OPT_PRECOMP_ORDER, OPT_SCANOV_V1, OPT_OV_PF, OPT_PRECOMP_G2REG,
  OPT_REFINE_COOP, OPT_PRECOMP_COMPACT, OPT_PREP_COOP, OPT_POOL_SORT_MEM, OPT_REFINE_SMALL, OPT_FINAL_ROUNDS,
  OPT_RANK_CT, OPT_RANK_WIN, OPT_RANK_SORT_NT, OPT_RANK_SORT_SMALL,
  OPT_COUNT
};
int64_t opt(Opt id, int64_t dflt);
inline bool opt_on(Opt id) { return opt(id, 0) != 0; }

inline bool is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }
inline int ilog2(int64_t n) { int k = 0; while ((int64_t(1) << k) < n) ++k; return k; }

// number of workgroups to launch for a persistent grid-stride kernel
int persistent_grid(const void* kernel, int block, size_t dyn_lds, int64_t work_items);

// ------------------------------------------------------------------------------------------------
// Hilbert curve (reference core/hilbert_mapper.py)
// ------------------------------------------------------------------------------------------------
__host__ __device__ constexpr inline void d2xy(uint32_t n, uint32_t idx, uint32_t& x_out, uint32_t& y_out) {
  // _hilbert_index_to_xy (:42-66) with _rotate (:92-113)
  uint32_t x = 0, y = 0, t = idx;
  for (uint32_t s = 1; s < n; s <<= 1) {
    uint32_t rx = 1u & (t >> 1);
    uint32_t ry = 1u & (t ^ rx);
    if (ry == 0) {
      if (rx == 1) { x = s - 1 - x; y = s - 1 - y; }
      uint32_t tmp = x; x = y; y = tmp;
    }
    x += s * rx;
    y += s * ry;
    t >>= 2;
  }
  x_out = x; y_out = y;
}

// Group LUT: float4 group j (Hilbert elements 4j..4j+3) is the 2x2 block at row-major offset
// `off` of an NS x NS image (layout invariant).  Entry = off | code << 16 where code
// holds, per element m, its slot b = (x & 1) + 2 (y & 1) inside the block (INV = false), or per
// slot b the element m it holds (INV = true).  Evaluated at compile time: a wave reads its entries
// from L2 instead of building the table per workgroup.
template <int NS>
struct GroupLut {
  uint32_t v[NS * NS / 4];
};
template <int NS, bool INV>
constexpr GroupLut<NS> make_group_lut() {
  GroupLut<NS> t{};
  for (uint32_t j = 0; j < (uint32_t)(NS * NS / 4); ++j) {
    uint32_t code = 0, off = 0;
    for (uint32_t m = 0; m < 4; ++m) {
      uint32_t x = 0, y = 0;
      d2xy(NS, 4 * j + m, x, y);
      if (m == 0) off = (y & ~1u) * NS + (x & ~1u);
      const uint32_t b = (x & 1u) + 2u * (y & 1u);
      code |= INV ? (m << (2 * b)) : (b << (2 * m));
    }
    t.v[j] = off | (code << 16);
  }
  return t;
}

// Scatter LUT of the chunk kernels: for every 2x2 group j (Hilbert positions 4j .. 4j + 3) the LDS byte
// offsets of its four values in the row-major n x n float image, two per dword (value m of the group in
// dword 2j + (m >> 1), bits 16 (m & 1) ..): one mask or shift per value gives the store address.
template <int NS>
struct alignas(16) AddrLut {  // read as uint4 by k_chunk_np
  uint32_t v[NS * NS / 2];
};
template <int NS>
constexpr AddrLut<NS> make_addr_lut() {
  AddrLut<NS> t{};
  for (uint32_t d = 0; d < (uint32_t)(NS * NS); ++d) {
    uint32_t x = 0, y = 0;
    d2xy(NS, d, x, y);
    t.v[d >> 1] |= (4u * (y * NS + x)) << (16 * (d & 1u));
  }
  return t;
}

__host__ __device__ inline uint32_t xy2d(uint32_t n, uint32_t x, uint32_t y) {
  // _xy_to_hilbert_index (:68-90); the rotate uses the loop's s, values wrap in uint32 which only
  // disturbs bits at or above s — never looked at again (SURVEY.md §8a note).
  uint32_t d = 0;
  for (uint32_t s = n >> 1; s > 0; s >>= 1) {
    uint32_t rx = (x & s) ? 1u : 0u;
    uint32_t ry = (y & s) ? 1u : 0u;
    d += s * s * ((3u * rx) ^ ry);
    if (ry == 0) {
      if (rx == 1) { x = s - 1 - x; y = s - 1 - y; }
      uint32_t tmp = x; x = y; y = tmp;
    }
  }
  return d;
}

// ------------------------------------------------------------------------------------------------
// streaming index schedule (core/streaming_index_builder.py:154-243)
// level l of a n*n stream has (n*n) >> (2l) values while l < max_levels (10)
// ------------------------------------------------------------------------------------------------
constexpr int kStreamMaxLevels = 10;

struct StreamSchedule {
  int nlev;                       // number of non-empty levels
  int64_t size[kStreamMaxLevels];
  int64_t alloc[kStreamMaxLevels];
  int64_t take[kStreamMaxLevels];  // values this level contributes (alloc if size > alloc else size)
  int64_t first[kStreamMaxLevels]; // output slot of this level's first value
  int64_t produced;                // total produced before truncation/padding to L
};

__host__ __device__ inline void stream_schedule(int64_t stream_len, int64_t L, StreamSchedule& s) {
  s.nlev = 0;
  int64_t sz = stream_len;
  while (s.nlev < kStreamMaxLevels && sz > 0) {
    s.size[s.nlev++] = sz;
    sz >>= 2;  // only full groups of 4 promote (:94)
  }
  int64_t remaining = L;
  int64_t out = 0;
  for (int i = 0; i < s.nlev; ++i) {
    int64_t a;
    if (i == s.nlev - 1) {
      a = remaining;
    } else {
      double frac = 1.0;
      for (int k = 0; k <= i; ++k) frac *= 0.5;  // 0.5 ** (i+1), exact
      a = (int64_t)((double)L * frac);
      if (a < 1) a = 1;
      if (a > remaining) a = remaining;
      remaining -= a;
    }
    s.alloc[i] = a;
    s.take[i] = (a <= 0) ? 0 : (s.size[i] > a ? a : s.size[i]);
    s.first[i] = out;
    out += s.take[i];
  }
  s.produced = out;
}

// output slot i -> (level, position); returns false for zero padding (:197-201)
__host__ __device__ inline bool stream_sample(const StreamSchedule& s, int64_t i, int& lev, int64_t& pos) {
  if (i >= s.produced) return false;
  for (int l = 0; l < s.nlev; ++l) {
    if (i < s.first[l] + s.take[l]) {
      int64_t k = i - s.first[l];
      lev = l;
      if (s.size[l] > s.alloc[l]) {
        double step = (double)s.size[l] / (double)s.alloc[l];  // len(level) / allocation (:187)
        pos = (int64_t)((double)k * step);                         // int(i * step) (:188)
      } else {
        pos = k;
      }
      return true;
    }
  }
  return false;
}

// ------------------------------------------------------------------------------------------------
// search level structure (core/search_engine.py:42-109)
// ------------------------------------------------------------------------------------------------
constexpr int kMaxSeg = 16;
struct SegTable {
  int nseg;
  int32_t grid[kMaxSeg];
  int32_t start[kMaxSeg];
  int32_t end[kMaxSeg];
  int32_t offset[kMaxSeg];
};

__host__ __device__ inline int isqrt_floor(int64_t v) {
  // int(math.sqrt(v)) for the small v used here
  int64_t r = (int64_t)sqrt((double)v);
  while (r * r > v) --r;
  while ((r + 1) * (r + 1) <= v) ++r;
  return (int)r;
}

__host__ __device__ inline void parse_structure(int64_t total, int64_t length, SegTable& t) {
  t.nseg = 0;
  if (length == 0 || total <= 0) return;
  int64_t remaining = total, cur = 0;
  int max_grid = isqrt_floor(total);
  if (max_grid > 32) max_grid = 32;
  int64_t g = 1;
  while (g <= max_grid) g *= 2;
  g /= 2;
  if (g < 2) g = 2;
  double frac = 0.5;
  uint64_t seen = 0;  // grids are powers of two <= 32 -> bit set by log2
  while (remaining > 0 && g >= 1 && cur < length) {
    int64_t a = (int64_t)((double)remaining * frac);
    if (g * g < a) a = g * g;
    if (remaining < a) a = remaining;
    if (a > 0 && t.nseg < kMaxSeg) {
      int lg = 0; while ((int64_t(1) << lg) < g) ++lg;
      t.grid[t.nseg] = (int32_t)g;
      t.start[t.nseg] = (int32_t)cur;
      t.end[t.nseg] = (int32_t)(cur + a);
      t.offset[t.nseg] = (seen >> lg) & 1;
      seen |= (uint64_t(1) << lg);
      t.nseg++;
      cur += a;
      remaining -= a;
    }
    g /= 2;
    frac *= 0.5;
    if (frac < 0.01) break;
  }
  if (remaining > 0 && cur < length && t.nseg > 0 && t.nseg < kMaxSeg) {
    t.grid[t.nseg] = t.grid[0];
    t.start[t.nseg] = (int32_t)cur;
    t.end[t.nseg] = (int32_t)((cur + remaining) < length ? (cur + remaining) : length);
    t.offset[t.nseg] = 1;
    t.nseg++;
  }
}

// ------------------------------------------------------------------------------------------------
// NumPy pairwise summation (numpy/_core/src/umath/loops_utils.h.src `pairwise_sum`), exact order:
//   n < 8: sequential from -0.0;  n <= 128: eight strided accumulators combined
//   ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then a sequential tail;  else split at n/2 rounded down to
//   a multiple of 8 and add the two halves.  np.add.reduce adds the identity first: 0 + pairwise.
// `f(k)` returns element k in the accumulation type T.  The split levels are separate non-inlined
// instantiations (no true recursion), bounded at 10 levels (n < 128 * 2^10).
// ------------------------------------------------------------------------------------------------
template <typename T, class F>
__device__ __forceinline__ T pw_leaf(const F& f, int off, int n) {
  if (n < 8) {
    T res = T(-0.0);
    for (int i = 0; i < n; ++i) res = res + f(off + i);
    return res;
  }
  T r0 = f(off), r1 = f(off + 1), r2 = f(off + 2), r3 = f(off + 3);
  T r4 = f(off + 4), r5 = f(off + 5), r6 = f(off + 6), r7 = f(off + 7);
  int i = 8;
  const int lim = n - (n % 8);
  for (; i < lim; i += 8) {
    r0 = r0 + f(off + i); r1 = r1 + f(off + i + 1); r2 = r2 + f(off + i + 2); r3 = r3 + f(off + i + 3);
    r4 = r4 + f(off + i + 4); r5 = r5 + f(off + i + 5); r6 = r6 + f(off + i + 6); r7 = r7 + f(off + i + 7);
  }
  T res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res = res + f(off + i);
  return res;
}

template <int D, typename T, class F>
__device__ __noinline__ T pw_rec(const F& f, int off, int n) {
  if constexpr (D == 0) {
    return pw_leaf<T>(f, off, n);
  } else {
    if (n <= 128) return pw_leaf<T>(f, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    T a = pw_rec<D - 1, T>(f, off, n2);
    T b = pw_rec<D - 1, T>(f, off + n2, n - n2);
    return a + b;
  }
}

// SM = true: the caller guarantees n <= 128 (no out-of-line split levels: a kernel without calls keeps
// its registers and needs no stack)
template <typename T, bool SM = false, class F>
__device__ __forceinline__ T np_sum(const F& f, int n) {
  if constexpr (SM) {
    return T(0) + pw_leaf<T>(f, 0, n);
  } else {
    if (n <= 128) return T(0) + pw_leaf<T>(f, 0, n);
    return T(0) + pw_rec<10, T>(f, 0, n);
  }
}

// Two sums over the same elements in one pass: np_sum<Sum2<T>>(f, n) with f(k) = {a_k, b_k} runs the
// pairwise order above on each component separately (component-wise +, no cross terms), so .a and .b
// are bit-identical to two np_sum<T> calls while every element is loaded once
template <typename T>
struct Sum2 {
  T a, b;
  __device__ __forceinline__ Sum2() = default;
  __device__ __forceinline__ Sum2(T a_, T b_) : a(a_), b(b_) {}
  __device__ __forceinline__ explicit Sum2(T v) : a(v), b(v) {}
  __device__ __forceinline__ Sum2 operator+(const Sum2& o) const { return Sum2(a + o.a, b + o.b); }
};

// element size of an HQ dtype code (0 if unknown)
inline int dtype_size(int dt) {
  switch (dt) {
    case HQ_U8: case HQ_I8: return 1;
    case HQ_F16: case HQ_I16: case HQ_BF16: return 2;
    case HQ_F32: case HQ_I32: return 4;
    case HQ_F64: case HQ_I64: return 8;
    default: return 0;
  }
}

// wave64 all-reduce through DPP (xor 1, xor 2, half-row mirror, row mirror) and four readlanes: no
// LDS round trips on the per-embedding critical path
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lanef(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wmin64(float v) {
  v = fminf(v, dppf<0xB1>(v));
  v = fminf(v, dppf<0x4E>(v));
  v = fminf(v, dppf<0x141>(v));
  v = fminf(v, dppf<0x140>(v));
  return fminf(fminf(lanef(v, 0), lanef(v, 16)), fminf(lanef(v, 32), lanef(v, 48)));
}
__device__ __forceinline__ float wmax64(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  return fmaxf(fmaxf(lanef(v, 0), lanef(v, 16)), fmaxf(lanef(v, 32), lanef(v, 48)));
}
// broadcast lane k of each 16-lane row (DPP row_newbcast)
template <int K>
__device__ __forceinline__ float rbc(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + K, 0xF, 0xF, false));
}

template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ int wsum64i(int v) {
  v += dppi<0xB1>(v);
  v += dppi<0x4E>(v);
  v += dppi<0x141>(v);
  v += dppi<0x140>(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
// Fast form of qz: with d = fl(x - mn) >= 0 (shared by both forms), the reference's
// y = fl(fl(d / rng) * 255) = Y (1+e1)(1+e2) and y' = fl(fl(d * fl(1/rng)) * 255) = Y (1+e3)(1+e4)(1+e5)
// with Y = 255 d / rng <= 255 and |ei| <= 2^-24, so |y - y'| <= 255 * 5 * 2^-24 < 7.7e-5 (with the
// hardware reciprocal, 1 ulp: |e3| <= 2^-23 and |y - y'| <= 255 * 6 * 2^-24 < 9.2e-5).  Hence
// trunc(y') == trunc(y) whenever frac(y') lies in [1e-4, 1 - 1e-4] (frac is exact: y' - floor(y')
// for y' < 2^23); otherwise `slow` is set and the caller recomputes that element with the exact
// division.
__device__ __forceinline__ uint32_t qfast(float x, float mn, float rcp, bool& slow) {
  const float y = ((x - mn) * rcp) * 255.0f;
  const float fl = floorf(y);
  const float f = y - fl;
  slow |= (f < 1e-4f) | (f > 0.9999f);
  return (uint32_t)fl;
}

}  // namespace hq
