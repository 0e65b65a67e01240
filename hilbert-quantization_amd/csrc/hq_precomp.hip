// hq_precomp.hip — pre-computed overlapping-square Hilbert index.
//
// Reference: core/precomputed_hilbert_index.py
//   :121-149 _calculate_granularity_levels  (square 2, 4, ... <= n/2, at most 6 levels, then (1, n))
//   :151-212 _precompute_level_averages     (grid squares row-major, then the (g-1)^2 squares offset
//                                            by half a square; float(np.mean(square)) -> float32)
//   :411-466 _compare_precomputed_levels    (float32 correlation + distance similarity)
//   :358-409 _calculate_precomputed_similarity (normalised level weights 0.4, 0.3, 0.2, 0.1, ...)
// HilbertQuantizer.quantize builds this index for every model (api.py:162-173).
//
// np.mean over a square is NumPy's pairwise sum over the C-order-flattened square (hq_common.h
// np_sum), so every average is bit-identical.  Squares of <= 128 values are one pairwise leaf (one
// thread); larger squares (16 x 16 and up: powers of two) split into 128-value leaves whose partial
// sums combine in a balanced binary tree — exactly NumPy's recursion for power-of-two lengths.
//
// One 256-thread workgroup per image: the image (or the Hilbert scatter of a 1-D parameter stream)
// is staged in LDS, leaf sums and averages stay in LDS, and the T averages leave with coalesced
// stores.
#include "hq_common.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace hq {

constexpr int kPreMaxLevels = 8;

__device__ constexpr GroupLut<16> kPreLut16 = make_group_lut<16, false>();
__device__ constexpr GroupLut<32> kPreLut32 = make_group_lut<32, false>();
__device__ constexpr GroupLut<64> kPreLut64 = make_group_lut<64, false>();
constexpr int kPreThreads = 256;

struct PreLevel {
  int g, s, count, off;  // grid side, square side, squares, first output
  int lsh;               // log2(s)
  int leaf0;             // first leaf task of this level (levels with s*s > 128)
  // zero-padding skip (1-D streams of d < n*n values): squares that touch a value < d, their list
  // offset in LDS and, for leaf levels, the first leaf task over the listed squares
  int zcnt, zoff, zleaf0;
};
struct PrePlan {
  int nlev, total, n_small, nleaves, lsh_n;
  int maxper;    // most 128-value leaves in one square
  int tree_lds;  // 1: combine the leaves through LDS (squares of > 64 leaves, or HQ_PRECOMP_TREE=lds)
  int diag;      // A/B diagnostics only (wrong averages): bit 0 skip small squares, 1 leaves, 2 load, 3 store
  int nt;        // non-temporal output stores
  int znz;       // zero-padding skip: squares listed over all levels (LDS list entries)
  int znleaves;  // zero-padding skip: leaf tasks over the listed squares
  int nleaves_al;  // LDS-tree partials rounded up so that res stays 16-byte aligned
  int leaf_rot;    // skip runs: leaf tasks from wave 1 when they fit three waves (pre_leaf_task)
  int g2reg;       // k_precomp_ws: the 2 x 2 grid squares (= Hilbert groups) averaged in the loader's
                   // registers, not listed; g2lvl = their level (-1: none)
  int g2lvl;
  PreLevel lv[kPreMaxLevels];
};

// host: levels of _calculate_granularity_levels (max_levels, min_square_size as the reference's
// defaults 6 and 2), outputs and leaf tasks
static int pre_plan(int n, int max_levels, int min_sq, PrePlan& p) {
  p.nlev = 0;
  p.total = 0;
  p.n_small = 0;
  p.nleaves = 0;
  p.maxper = 0;
  p.tree_lds = 0;
  p.diag = 0;
  p.nt = 1;
  p.lsh_n = ilog2(n);
  int s = min_sq;
  int lv_g[16], lv_s[16], c = 0;
  while (s <= n / 2 && c < max_levels) {
    const int g = n / s;
    if (g >= 2) { lv_g[c] = g; lv_s[c] = s; ++c; }
    s *= 2;
  }
  if (c == 0 || lv_s[c - 1] < n) { lv_g[c] = 1; lv_s[c] = n; ++c; }
  if (c > kPreMaxLevels) return HQ_E_UNSUPPORTED;
  for (int i = 0; i < c; ++i) {
    PreLevel& L = p.lv[i];
    L.g = lv_g[i];
    L.s = lv_s[i];
    L.lsh = ilog2(L.s);
    if ((1 << L.lsh) != L.s) return HQ_E_UNSUPPORTED;
    L.count = L.g * L.g + (L.s / 2 > 0 ? (L.g - 1) * (L.g - 1) : 0);
    L.off = p.total;
    p.total += L.count;
    L.leaf0 = -1;
    if (L.s * L.s <= 128) {
      if (L.off != p.n_small) return HQ_E_UNSUPPORTED;  // small squares form a prefix (finest first)
      p.n_small += L.count;
    } else {
      const int per = L.s * L.s / 128;
      p.nleaves = (p.nleaves + per - 1) / per * per;  // a square's leaves start on a multiple of per
      L.leaf0 = p.nleaves;
      p.nleaves += L.count * per;
      if (per > p.maxper) p.maxper = per;
    }
  }
  p.nlev = c;
  if (2 * p.maxper > 64) p.tree_lds = 1;  // a square's leaf lanes would span waves
  p.nleaves_al = (p.nleaves + 3) & ~3;  // f64 partials: a multiple of 16 B already
  p.leaf_rot = 1;
  p.g2reg = 0;
  p.g2lvl = -1;
  for (int i = 0; i < p.nlev; ++i)
    if (p.lv[i].s == 2 && p.lv[i].leaf0 < 0) p.g2lvl = i;
  return HQ_OK;
}

// Zero-padding skip for a 1-D stream of d < n*n values (pipeline padding, core/pipeline.py:325-349):
// every cell at Hilbert index >= d is +0.0 in every image, so a square none of whose cells lies below
// d averages to exactly +0.0 (np.mean of zeros) and is never computed — its output slot is zeroed once
// per workgroup.  A square (aligned or offset by half a side) is the union of four aligned sub-blocks
// of side h = s/2, each a contiguous Hilbert range starting at a multiple of h^2 (layout invariant,
// SURVEY.md §8a); for h = 1 the test uses the sub-block's 2x2 group start 4j, a lower bound: a listed
// square may still be all zero (computed, exact), an unlisted one never holds data.  The host builds
// the lists (square indices per level, 16 bit) once per configuration (pre_zero_lists); returns 1
// when the skip removes squares.  lists (optional): the listed squares per level, ascending.
static int pre_zero_plan(int n, int d, PrePlan& p, std::vector<std::vector<int>>* lists = nullptr) {
  p.znz = 0;
  p.znleaves = 0;
  if (d >= n * n || n > 64) return 0;
  static thread_local uint16_t hidx[64 * 64];
  for (uint32_t i = 0; i < (uint32_t)(n * n); ++i) {
    uint32_t x, y;
    d2xy((uint32_t)n, i, x, y);
    hidx[y * n + x] = (uint16_t)i;
  }
  if (lists) lists->assign(p.nlev, {});
  for (int l = 0; l < p.nlev; ++l) {
    PreLevel& L = p.lv[l];
    const int h = L.s >> 1, lg = ilog2(L.g);
    L.zcnt = 0;
    L.zoff = p.znz;
    for (int k = 0; k < L.count; ++k) {
      int x0, y0;
      if (k < L.g * L.g) {
        y0 = (k >> lg) * L.s;
        x0 = (k & (L.g - 1)) * L.s;
      } else {
        const int kk = k - L.g * L.g, hw = L.g - 1;
        y0 = (kk / hw) * L.s + L.s / 2;
        x0 = (kk % hw) * L.s + L.s / 2;
      }
      bool nz = false;
      for (int q = 0; q < (h > 0 ? 4 : 1); ++q) {
        const int cx = x0 + (q & 1) * h, cy = y0 + (q >> 1) * h;
        int start = hidx[cy * n + cx] & ~3;
        if (h >= 2) start &= ~(h * h - 1);
        nz |= start < d;
      }
      if (p.g2reg && l == p.g2lvl && k < L.g * L.g) nz = false;  // averaged in the loader's registers
      L.zcnt += nz;
      if (nz && lists) (*lists)[l].push_back(k);
    }
    p.znz += L.zcnt;
    L.zleaf0 = -1;
    if (L.leaf0 >= 0) {
      const int per = L.s * L.s / 128;
      p.znleaves = (p.znleaves + per - 1) / per * per;
      L.zleaf0 = p.znleaves;
      p.znleaves += L.zcnt * per;
    }
  }
  if (2 * p.znleaves > kPreThreads || p.total > 4096) return 0;  // one leaf round
  return p.znz < p.total;
}

// Order of a small-square level's list for the LDS banks (f32 images, row stride ld): list position i
// is read by lane i mod 64 of its wave, and a wave-instruction's lanes are serviced in groups
// (MI355X_MICROARCH.md §LDS).  Per square size the reads are: 1 x 1 / 2 x 2 dword reads (two 32-lane
// groups, bank = dword mod 32), 4 x 4 two-dword pairs of ds_read2_b64 (16-lane groups, mod 32), 8 x 8
// ds_read_b128 (the four 16-lane groups of that instruction, mod 64).  A square's reads are its corner
// address plus offsets common to all lanes, so a group is conflict-free when its corners fall in
// distinct bank classes: greedily, each group takes one square from each of the fullest classes.
static void pre_bank_order(std::vector<int>& ks, const PreLevel& L, int ld) {
  const int cnt = (int)ks.size();
  if (cnt < 2 || L.s > 8) return;
  int ncls, div, mod;
  std::vector<std::vector<int>> groups;
  auto contiguous = [&](int gs) {
    for (int g0 = 0; g0 < 64; g0 += gs) {
      groups.push_back({});
      for (int l = g0; l < g0 + gs; ++l) groups.back().push_back(l);
    }
  };
  if (L.s <= 2) { ncls = 32; div = 1; mod = 32; contiguous(32); }
  else if (L.s == 4) { ncls = 16; div = 2; mod = 32; contiguous(16); }
  else {
    ncls = 16; div = 4; mod = 64;
    // ds_read_b128 lane groups: {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32
    for (int hh = 0; hh < 64; hh += 32) {
      std::vector<int> g1, g2;
      for (int l = 0; l < 4; ++l) g1.push_back(hh + l);
      for (int l = 12; l < 16; ++l) g1.push_back(hh + l);
      for (int l = 20; l < 28; ++l) g1.push_back(hh + l);
      for (int l = 4; l < 12; ++l) g2.push_back(hh + l);
      for (int l = 16; l < 20; ++l) g2.push_back(hh + l);
      for (int l = 28; l < 32; ++l) g2.push_back(hh + l);
      groups.push_back(g1);
      groups.push_back(g2);
    }
  }
  std::vector<std::vector<int>> bucket(ncls);
  const int lg = ilog2(L.g);
  for (int k : ks) {
    int x0, y0;
    if (k < L.g * L.g) {
      y0 = (k >> lg) * L.s;
      x0 = (k & (L.g - 1)) * L.s;
    } else {
      const int kk = k - L.g * L.g, hw = L.g - 1;
      y0 = (kk / hw) * L.s + L.s / 2;
      x0 = (kk % hw) * L.s + L.s / 2;
    }
    bucket[((y0 * ld + x0) % mod) / div].push_back(k);
  }
  for (auto& b : bucket) std::reverse(b.begin(), b.end());  // pop_back yields ascending k
  std::vector<int> out(cnt, -1);
  for (int b0 = 0; b0 < cnt; b0 += 64) {
    for (const auto& g : groups) {
      std::vector<char> used(ncls, 0);
      for (int l : g) {
        if (b0 + l >= cnt) continue;
        int best = -1;
        for (int c = 0; c < ncls; ++c)  // the fullest class not yet in this group, else the fullest
          if (!bucket[c].empty() && (best < 0 || (used[best] && !used[c]) ||
                                     (used[best] == used[c] && bucket[c].size() > bucket[best].size())))
            best = c;
        used[best] = 1;
        out[b0 + l] = bucket[best].back();
        bucket[best].pop_back();
      }
    }
  }
  ks.swap(out);
}

// The lists of one configuration in device memory, built once (host) and cached for the process:
// per level at zoff, the listed squares (small levels in bank order for f32, leaf levels ascending).
// The first call per configuration allocates the buffer (hipMalloc: may synchronise the device, so a
// graph capture must not contain that first call) and uploads the list on the caller's stream; an event
// behind the upload is kept, and every call makes its stream wait on it (a no-op once it completed), so a
// launch on another stream never reads the list before it arrived.  The host copy stays with the cache
// entry (the asynchronous copy may read it after the call returns).
__host__ __device__ inline int pre_map_off(int znz) { return (znz + 7) & ~7; }

struct PreZeroList {
  uint16_t* dptr = nullptr;
  hipEvent_t ready = nullptr;
  std::vector<uint16_t> host;
};

static const uint16_t* pre_zero_lists(int n, int d, int ld, int esz, int max_levels, int min_sq, int order,
                                      const PrePlan& plan, hipStream_t s, int& err) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int, int>, PreZeroList*> cache;
  int dev = 0;
  err = HQ_OK;
  if (hipGetDevice(&dev) != hipSuccess) { err = HQ_E_HIP; return nullptr; }
  const auto key = std::make_tuple(dev, n, d, ld, esz, max_levels, min_sq, order, plan.g2reg);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) {
    if (hipStreamWaitEvent(s, it->second->ready, 0) != hipSuccess) { err = HQ_E_HIP; return nullptr; }
    return it->second->dptr;
  }
  PrePlan p = plan;
  std::vector<std::vector<int>> lists;
  pre_zero_plan(n, d, p, &lists);
  PreZeroList* e = new PreZeroList();
  for (int l = 0; l < p.nlev; ++l) {
    if (order && esz == 4 && p.lv[l].leaf0 < 0) pre_bank_order(lists[l], p.lv[l], ld);
    for (int k : lists[l]) e->host.push_back((uint16_t)k);
  }
  if ((int)e->host.size() != p.znz) { delete e; err = HQ_E_UNSUPPORTED; return nullptr; }
  // then, 16-byte aligned at pre_map_off(znz), the inverse map of the compact averages (k_precomp_ws<.., CMP>):
  // output slot o -> 1 + its list position (the average's LDS slot), 0 for a square of zero padding
  e->host.resize((size_t)pre_map_off(p.znz) + p.total, 0);
  for (int l = 0; l < p.nlev; ++l)
    for (size_t i = 0; i < lists[l].size(); ++i)
      e->host[pre_map_off(p.znz) + p.lv[l].off + lists[l][i]] = (uint16_t)(p.lv[l].zoff + i + 1);
  const size_t bytes = e->host.size() * sizeof(uint16_t);
  if (hipMalloc(&e->dptr, bytes + 16) != hipSuccess) { delete e; err = HQ_E_HIP; return nullptr; }
  if (hipMemcpyAsync(e->dptr, e->host.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipEventCreateWithFlags(&e->ready, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(e->ready, s) != hipSuccess) {
    (void)hipStreamSynchronize(s);  // the copy may be in flight: let it finish before freeing its buffers
    if (e->ready) (void)hipEventDestroy(e->ready);
    (void)hipFree(e->dptr);
    delete e;
    err = HQ_E_HIP;
    return nullptr;
  }
  cache[key] = e;
  return e->dptr;
}

// top-left corner of square k of a level (grid squares row-major, then offset squares).  g is a power
// of two (shifts); the offset grid's side g - 1 is not: its row is floor((k + 0.5) / (g - 1)) in f32,
// exact for n <= 128: k < 63^2 and g - 1 <= 63 put (k + 0.5) / (g - 1) (<= 63) at least 1/126 away
// from an integer, while v_rcp_f32 + the product err by < 63 * 2^-21.
__device__ __forceinline__ void pre_square(const PreLevel& L, int k, int& x0, int& y0) {
  const int lg = __builtin_ctz((unsigned)L.g);
  const int gg = L.g * L.g;
  if (k < gg) {
    y0 = (k >> lg) << L.lsh;
    x0 = (k & (L.g - 1)) << L.lsh;
  } else {
    k -= gg;
    const int h = L.g - 1;
    const int r = (int)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)h));
    y0 = (r << L.lsh) + L.s / 2;
    x0 = ((k - r * h) << L.lsh) + L.s / 2;
  }
}

// np.mean's f64 division by the count (_methods._mean; f32 input: f32(f64(sum) / cnt)).  Every count
// here is a power of two (s * s squares), so the division is the exact product with 1 / cnt: one
// rounding either way, and none at all before the final cast unless the result is subnormal.
template <typename T>
__device__ __forceinline__ float pre_mean(T s, int lcnt) {
  const double inv = __builtin_amdgcn_ldexp(1.0, -lcnt);  // 2^-lcnt, cnt = 2^lcnt
  return (float)((double)s * inv);
}

// eight consecutive values from a 16-byte aligned LDS address
template <typename T>
__device__ __forceinline__ void load8(const T* p, T (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const double2 a = *reinterpret_cast<const double2*>(p + 2 * h);
      v[2 * h] = a.x;
      v[2 * h + 1] = a.y;
    }
  }
}

// four consecutive values from a 16-byte aligned LDS address
template <typename T>
__device__ __forceinline__ void load4(const T* p, T (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
    const double2 a = *reinterpret_cast<const double2*>(p), b = *reinterpret_cast<const double2*>(p + 2);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
}

// np.add.reduce over an S x S square (S = 4 or 8: 16 / 64 values, one pairwise leaf) whose rows start
// at b, b + ld, ...: eight accumulators over the C-order flattening, then
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), identity added first.  Rows are read as S/2-wide vectors.
template <typename T, int S>
__device__ __forceinline__ T sq_sum(const T* b, int ld) {
  if constexpr (S == 8) {
    // 8x8: row r is step r of the eight accumulators; at most four rows of loads in flight (VGPRs)
    T r8[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      T v[8];
      load8<T>(b + r * ld, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) r8[j] = r == 0 ? v[j] : r8[j] + v[j];
      // rows 4-7 are addressed through a pointer that depends on the first four rows' sums, so no pass
      // can issue all 16 loads at once (64 VGPRs in flight)
      if (r == 3) {
        int z = 0;
        asm volatile("" : "+v"(z) : "v"(r8[0]), "v"(r8[4]));
        b += z;
      }
    }
    return T(0) + (((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7])));
  }
  T x[S * S];
#pragma unroll
  for (int r = 0; r < S; ++r)
#pragma unroll
    for (int c = 0; c < S; c += S / 2) {
      if constexpr (S == 8 && sizeof(T) == 4) {
        const float4 v = *reinterpret_cast<const float4*>(b + r * ld + c);
        x[r * S + c] = v.x; x[r * S + c + 1] = v.y; x[r * S + c + 2] = v.z; x[r * S + c + 3] = v.w;
      } else if constexpr (sizeof(T) == 4 || S == 4) {
        // 4x4 (two 8-byte halves per row) or 8x8 f64 (two 16-byte quarters per half row)
#pragma unroll
        for (int h = 0; h < S / 2; h += 2) {
          if constexpr (sizeof(T) == 4) {
            const float2 v = *reinterpret_cast<const float2*>(b + r * ld + c + h);
            x[r * S + c + h] = v.x; x[r * S + c + h + 1] = v.y;
          } else {
            const double2 v = *reinterpret_cast<const double2*>(b + r * ld + c + h);
            x[r * S + c + h] = v.x; x[r * S + c + h + 1] = v.y;
          }
        }
      } else {
#pragma unroll
        for (int h = 0; h < S / 2; h += 2) {
          const double2 v = *reinterpret_cast<const double2*>(b + r * ld + c + h);
          x[r * S + c + h] = v.x; x[r * S + c + h + 1] = v.y;
        }
      }
    }
  T r8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r8[j] = x[j];
#pragma unroll
  for (int i = 8; i < S * S; i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r8[j] = r8[j] + x[i + j];
  return T(0) + (((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7])));
}

// all squares of one level with S x S <= 128 values (S = 1, 2, 4, 8): one NumPy pairwise leaf per thread
template <typename T, int S, bool SK, bool CMP = false>
__device__ __forceinline__ void pre_small(const PreLevel& L, const T* img, int ld, float* res, int tid,
                                          const uint16_t* zl) {
  const int cnt = SK ? L.zcnt : L.count;
  for (int i = tid; i < cnt; i += kPreThreads) {
    int k;
    const T* b;
    if constexpr (SK) {
      k = zl[L.zoff + i];  // a listed square; its corner from the level geometry
      int x0, y0;
      pre_square(L, k, x0, y0);
      b = img + y0 * ld + x0;
    } else {
      k = i;
      int x0, y0;
      pre_square(L, k, x0, y0);
      b = img + y0 * ld + x0;
    }
    T sum;
    if constexpr (S == 8) sum = sq_sum<T, 8>(b, ld);
    else if constexpr (S == 4) sum = sq_sum<T, 4>(b, ld);
    else if constexpr (S == 2) sum = T(0) + ((((T(-0.0) + b[0]) + b[1]) + b[ld]) + b[ld + 1]);  // NumPy n < 8 branch
    else sum = T(0) + (T(-0.0) + b[0]);  // one value
    res[CMP ? L.zoff + i : L.off + k] = pre_mean<T>(sum, 2 * L.lsh);  // CMP: compact slot = list position
  }
}

// once per workgroup before the image loop (skip runs): the host-built lists of the squares that
// touch a value < d (pre_zero_lists) into LDS, then the image and the averages zeroed — the padding
// cells and the unlisted averages stay +0.0 for every image
template <typename T>
__device__ __forceinline__ void pre_zero_setup(T* img, float* res, uint16_t* zl, const uint16_t* __restrict__ glist,
                                               int znz, int total, int n, int ld, int tid) {
  for (int i = tid; i < znz; i += kPreThreads) zl[i] = glist[i];
  for (int i = tid; i < ld * n; i += kPreThreads) img[i] = T(0);
  for (int i = tid; i < total; i += kPreThreads) res[i] = 0.0f;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Skip runs: this thread's half-leaf task, fixed for the workgroup (one round, 2 * znleaves <= 256),
// resolved once after pre_zero_setup: lt_b = LDS offset of its first value; lt_m = the average's slot
// (bits 0-11), log2 of the square side (12-15), the leaf within the square (16-20), live (24)
// When the leaf tasks fit three waves they start at wave 1: the small-square levels fill waves from wave 0
// (the 8 x 8 squares, fewest, on wave 0 alone), so the waves' LDS work up to the image's barrier evens out.
__device__ __forceinline__ void pre_leaf_task(const PreLevel* lv, const PrePlan& plan, const uint16_t* zl, int ld,
                                              int tid, int& lt_b, int& lt_m, bool cmp = false) {
  const int rot = 2 * plan.znleaves <= kPreThreads - 64 && plan.leaf_rot ? 64 : 0;
  const int t = (tid - rot) >> 1;
  lt_b = 0;
  lt_m = 0;
  if (tid < rot || t >= plan.znleaves) return;
  int l = plan.nlev - 1;
  while (lv[l].zleaf0 < 0 || t < lv[l].zleaf0) --l;
  const int lper = 2 * lv[l].lsh - 7;  // log2 of the leaves per square
  const int slot = (t - lv[l].zleaf0) >> lper, leaf = (t - lv[l].zleaf0) & ((1 << lper) - 1);
  if (slot >= lv[l].zcnt) return;  // an alignment gap before the next level
  const int k = zl[lv[l].zoff + slot];
  int x0, y0;
  pre_square(lv[l], k, x0, y0);
  lt_b = y0 * ld + x0 + 4 * (tid & 1);
  lt_m = (cmp ? lv[l].zoff + slot : lv[l].off + k) | (lv[l].lsh << 12) | (leaf << 16) | (1 << 24);
}

// squares of <= 128 values: one thread each, level by level (uniform geometry per loop); 4x4 and 8x8
// squares read whole row segments (their x0 is a multiple of s/2) and sum in registers
template <typename T, bool SK, bool CMP = false>
__device__ __forceinline__ void pre_small_levels(const PreLevel* lv, int nlev, const T* img, int ld, float* res,
                                                 int tid, const uint16_t* zl) {
  for (int l = 0; l < nlev; ++l) {
    // this level's geometry from the LDS copy into SGPRs (indexing the kernarg plan by a loop variable
    // keeps the whole plan live in SGPRs, which spill)
    PreLevel L;
    L.g = __builtin_amdgcn_readfirstlane(lv[l].g);
    L.s = __builtin_amdgcn_readfirstlane(lv[l].s);
    L.count = __builtin_amdgcn_readfirstlane(lv[l].count);
    L.off = __builtin_amdgcn_readfirstlane(lv[l].off);
    L.lsh = __builtin_amdgcn_readfirstlane(lv[l].lsh);
    L.leaf0 = __builtin_amdgcn_readfirstlane(lv[l].leaf0);
    if (L.leaf0 >= 0) continue;
    // one straight-line loop per square size (the size is uniform per level)
    L.zcnt = __builtin_amdgcn_readfirstlane(lv[l].zcnt);
    L.zoff = __builtin_amdgcn_readfirstlane(lv[l].zoff);
    if (L.s == 2) pre_small<T, 2, SK, CMP>(L, img, ld, res, tid, zl);
    else if (L.s == 4) pre_small<T, 4, SK, CMP>(L, img, ld, res, tid, zl);
    else if (L.s == 8) pre_small<T, 8, SK, CMP>(L, img, ld, res, tid, zl);
    else pre_small<T, 1, SK, CMP>(L, img, ld, res, tid, zl);
  }
}

// Skip runs: 128-value leaves of the larger squares from the task resolved once per workgroup (lt_b: LDS
// offset of the half leaf's first value; lt_m: average slot bits 0-11, log2 side 12-15, leaf 16-20, live
// 24).  Two lanes per leaf: lane h = 0 / 1 keeps NumPy's accumulators r0-r3 / r4-r7 (columns 4h..4h+3 of
// each 8-value step, 16 steps of one row segment), so ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)) is one
// shuffle; a square's leaves sit on consecutive lanes of one wave and combine in NumPy's balanced tree.
template <typename T>
__device__ __forceinline__ void pre_leaves_sk(const T* img, int ld, float* res, int tid, int lt_b, int lt_m,
                                              int maxper) {
  const int h = tid & 1;
  // laundered per image: hoisted out of the image loop, the 16 load addresses would hold VGPRs
  asm volatile("" : "+v"(lt_b), "+v"(lt_m));
  const bool live = (lt_m >> 24) & 1;
  const int lsh = (lt_m >> 12) & 15, leaf = (lt_m >> 16) & 31;
  T v = T(0);
  if (live) {
    const T* b = img + lt_b;
    const int msk = (1 << lsh) - 1;
    T r[4];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int q = (leaf << 7) + 8 * i;
      T w4[4];
      load4<T>(b + (q >> lsh) * ld + (q & msk), w4);
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = i == 0 ? w4[j] : r[j] + w4[j];
      if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // at most 8 steps of loads in flight
    }
    v = (r[0] + r[1]) + (r[2] + r[3]);
  }
  const int per = live ? 1 << (2 * lsh - 7) : 0;
  {
    const T o = __shfl_down(v, 1, 64);
    if (h == 0) v = v + o;
  }
  for (int w = 1; w < maxper; w <<= 1) {
    const T o = __shfl_down(v, 2 * w, 64);
    if (w < per && h == 0 && (leaf & (2 * w - 1)) == 0) v = v + o;
  }
  if (live && h == 0 && leaf == 0) res[lt_m & 0xFFF] = pre_mean<T>(T(0) + v, 2 * lsh);
}

// The T averages from LDS to the output row o by threads t0 = 0 .. nthr-1: float4 stores from the row's
// first 16-byte boundary; for 8-B aligned rows (even strides) the float4 comes from two 8-byte LDS reads
// (2-way bank conflicts at the 16-B lane stride: 8 LDS cycles per wave, where two 4-way ds_read2_b32
// took 32), else from dword reads; scalar head and tail.  nt: non-temporal (written once).
__device__ __forceinline__ void pre_store(const float* res, int total, float* o, bool nt, int t0, int nthr) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef float f2v __attribute__((ext_vector_type(2)));
  const int mis = (int)((reinterpret_cast<uintptr_t>(o) >> 2) & 3);
  const int head = min((4 - mis) & 3, total);
  const int nv = (total - head) >> 2;
  if (t0 < head) o[t0] = res[t0];
  for (int i = t0; i < nv; i += nthr) {
    const int a = head + 4 * i;
    f4v v;
    if (!(mis & 1)) {
      // volatile: two ds_read_b64, not one merged ds_read2_b64 (its 16-lane groups conflict 2-way too)
      typedef __attribute__((address_space(3))) const volatile f2v lds_f2v;
      const f2v lo = *(lds_f2v*)(res + a);
      const f2v hi = *(lds_f2v*)(res + a + 2);
      v = f4v{lo.x, lo.y, hi.x, hi.y};
    } else {
      v = f4v{res[a], res[a + 1], res[a + 2], res[a + 3]};
    }
    if (nt) __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(o + a));
    else *reinterpret_cast<f4v*>(o + a) = v;
  }
  for (int a = head + 4 * nv + t0; a < total; a += nthr) o[a] = res[a];
}

// pre_store for compact averages (k_precomp_ws<.., CMP>): output slot a holds res[map[a] - 1], or +0.0 where
// map[a] == 0 (a square of zero padding: np.mean of zeros).  The storer waves issue no global loads in the
// image loop (on gfx9 a load's wait would also wait for the wave's older stores), so the map entries of a
// lane's slots live in registers: PreMapRegs::load reads them for one row alignment (the float4 groups start
// at the row's first 16-byte boundary) and is re-run only when a row's alignment differs from the last one.
constexpr int kPreStoreG = 6;  // float4 groups per storer lane (128 lanes): total <= 3072 averages
struct PreMapRegs {
  uint32_t m[kPreStoreG][2];
  uint32_t ht;  // head slot (lane < head) in the low half, tail slot (lane < tail count) in the high half
  int mis;
  __device__ __forceinline__ void load(const uint16_t* __restrict__ map, int total, int mis_, int t0, int nthr) {
    mis = mis_;
    const int head = min((4 - mis) & 3, total);
    const int nv = (total - head) >> 2;
#pragma unroll
    for (int j = 0; j < kPreStoreG; ++j) {
      const int i = t0 + nthr * j;
      const int a = head + 4 * i;
      m[j][0] = m[j][1] = 0u;
      if (i < nv) {
        m[j][0] = (uint32_t)map[a] | ((uint32_t)map[a + 1] << 16);
        m[j][1] = (uint32_t)map[a + 2] | ((uint32_t)map[a + 3] << 16);
      }
    }
    const int ta = head + 4 * nv + t0;
    ht = (t0 < head ? (uint32_t)map[t0] : 0u) | ((ta < total ? (uint32_t)map[ta] : 0u) << 16);
  }
};

__device__ __forceinline__ void pre_store_map(const float* res, const PreMapRegs& mr, int total, float* o, bool nt,
                                              int t0, int nthr) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  auto val = [&](uint32_t m) -> float { return m ? res[m - 1] : 0.0f; };
  const int head = min((4 - mr.mis) & 3, total);
  const int nv = (total - head) >> 2;
  if (t0 < head) o[t0] = val(mr.ht & 0xFFFFu);
#pragma unroll
  for (int j = 0; j < kPreStoreG; ++j) {
    const int i = t0 + nthr * j;
    if (i < nv) {
      const int a = head + 4 * i;
      const f4v v = f4v{val(mr.m[j][0] & 0xFFFFu), val(mr.m[j][0] >> 16), val(mr.m[j][1] & 0xFFFFu),
                        val(mr.m[j][1] >> 16)};
      if (nt) __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(o + a));
      else *reinterpret_cast<f4v*>(o + a) = v;
    }
  }
  const int ta = head + 4 * nv + t0;
  if (ta < total) o[ta] = val(mr.ht >> 16);
}

// phase-skipping diagnostics (wrong averages): `make DIAG=1` builds only
#ifdef HQ_DIAG
#define PRE_DIAG(bit) (plan.diag & (bit))
#else
#define PRE_DIAG(bit) false
#endif

// kind 0: images (n x n row-major, image stride `stride` elements); kind 1: 1-D Hilbert-ordered
// parameter streams of d values (row stride `stride`), zero-padded to n*n and mapped to 2-D
// (core/pipeline.py:298-319 _get_2d_representation).
template <typename T, int PF, bool SK, int KG>
__global__ __launch_bounds__(kPreThreads) __attribute__((amdgpu_waves_per_eu(5))) void k_precomp(const T* __restrict__ in, int kind, int64_t N, int64_t stride,
                                                         int d, int n, PrePlan plan, float* __restrict__ out,
                                                         int64_t out_stride, int use_lut, int ld,
                                                         const uint16_t* __restrict__ glist) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ PreLevel lv[kPreMaxLevels];  // per-thread level lookups index LDS, not the kernarg block
  T* img = reinterpret_cast<T*>(smem);
  T* part = img + ((ld * n + 3) & ~3);  // row stride ld = n + pad (16-B aligned rows spread the bank pattern)
  float* res = reinterpret_cast<float*>(part + (plan.tree_lds ? plan.nleaves_al : 0));  // part: LDS tree only; res 16-B aligned
  uint16_t* zl = reinterpret_cast<uint16_t*>(res + ((plan.total + 3) & ~3));  // SK: listed squares, per level at zoff
  const int tid = threadIdx.x;
  const int lsh_n = plan.lsh_n;
  // skip runs are 1-D streams with the group LUT (host): the other load paths are compiled out, so
  // their loads cannot hold back the wait counters of this one
  const bool lut_on = SK || use_lut;
  const int knd = SK ? 1 : kind;
  if (tid < plan.nlev) lv[tid] = plan.lv[tid];
  // The barriers below order LDS only: s_waitcnt lgkmcnt(0) + s_barrier, so the prefetch of the next
  // image (plain global loads into registers) stays in flight through this image's reductions
  // (__syncthreads' release fence would wait for it with vmcnt(0)).
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  // 1-D streams with the compile-time group LUT (n = 16 / 32 / 64): each thread owns float4 groups
  // j = tid + 256 i (2x2 blocks, Hilbert layout invariant); their LUT entries live in registers and
  // the next image's values are fetched while the current one is reduced
  constexpr int kPreG = KG;  // groups per thread: 4 at n = 64; 2 when a skip run reads only d <= 2048 values
  const int G = (n * n) >> 2;
  uint32_t lut[kPreG];
  T pf[kPreG][4];
  if (lut_on) {
    const uint32_t* glut = n == 16 ? kPreLut16.v : (n == 32 ? kPreLut32.v : kPreLut64.v);
#pragma unroll
    for (int i = 0; i < kPreG; ++i) lut[i] = tid + kPreThreads * i < G ? glut[tid + kPreThreads * i] : 0u;
  }
  // The per-thread group geometry (element masks against d, LUT scatter offsets) is loop-invariant;
  // hoisted out of the image loop it held ~40 VGPRs and spilled SGPR masks, so it is laundered per
  // image (empty asm) and recomputed: a few VALU ops against a wave per SIMD more.
  auto fetch = [&](int64_t e) {
    const T* src = in + e * stride;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
    int dd = d;
    asm volatile("" : "+s"(dd));
#pragma unroll
    for (int i = 0; i < kPreG; ++i) {
      const int j = tid + kPreThreads * i;
      const int d = dd;
      if (vec_ok && 4 * j + 3 < d) {
        if constexpr (sizeof(T) == 4) {
          const float4 q4 = *reinterpret_cast<const float4*>(src + 4 * j);
          pf[i][0] = q4.x; pf[i][1] = q4.y; pf[i][2] = q4.z; pf[i][3] = q4.w;
        } else {
          const double2 a2 = *reinterpret_cast<const double2*>(src + 4 * j);
          const double2 b2 = *reinterpret_cast<const double2*>(src + 4 * j + 2);
          pf[i][0] = a2.x; pf[i][1] = a2.y; pf[i][2] = b2.x; pf[i][3] = b2.y;
        }
      } else {
#pragma unroll
        for (int m = 0; m < 4; ++m) pf[i][m] = 4 * j + m < d ? src[4 * j + m] : T(0);  // zero padding
      }
    }
  };
  int lt_b = 0, lt_m = 0;
  if constexpr (SK) {
    pre_zero_setup<T>(img, res, zl, glist, plan.znz, plan.total, n, ld, tid);
    pre_leaf_task(lv, plan, zl, ld, tid, lt_b, lt_m);
  }
  if (PF && lut_on && (int64_t)blockIdx.x < N) fetch(blockIdx.x);
  for (int64_t e = blockIdx.x; e < N; e += gridDim.x) {
    const T* src = in + e * stride;
    if (PRE_DIAG(4)) {
    } else if (knd == 0) {
      for (int i = tid; i < n * n; i += kPreThreads) img[(i >> lsh_n) * ld + (i & (n - 1))] = src[i];
    } else if (lut_on) {
      if (!PF) fetch(e);
#pragma unroll
      for (int i = 0; i < kPreG; ++i) {
        if (tid + kPreThreads * i >= G) continue;
        if constexpr (SK) {  // all padding: stays +0.0 from the setup (bound laundered per image, as in fetch)
          int dz = d;
          asm volatile("" : "+s"(dz));
          if (4 * (tid + kPreThreads * i) >= dz) continue;
        }
        uint32_t ent = lut[i];
        asm volatile("" : "+v"(ent));
        const uint32_t off0 = ent & 0xFFFFu, code = ent >> 16;
        const uint32_t off = (off0 >> lsh_n) * ld + (off0 & (n - 1));
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t b = (code >> (2 * m)) & 3u;
          img[off + (b & 1u) + (b >> 1) * ld] = pf[i][m];
        }
      }
    } else {
      for (int i = tid; i < n * n; i += kPreThreads) {
        uint32_t x, y;
        d2xy((uint32_t)n, (uint32_t)i, x, y);
        img[y * ld + x] = i < d ? src[i] : T(0);
      }
    }
    lds_barrier();
    if (PF && lut_on && e + gridDim.x < N) fetch(e + gridDim.x);
    // squares of <= 128 values: one thread each, level by level (uniform geometry per loop); 4x4 and
    // 8x8 squares read whole row segments (their x0 is a multiple of s/2) and sum in registers
    if (!PRE_DIAG(1)) pre_small_levels<T, SK>(lv, plan.nlev, img, ld, res, tid, zl);
    // 128-value leaves of the larger squares: 16 steps of 8 consecutive values (one row segment,
    // 8-aligned because x0 is a multiple of s/2 >= 8), eight accumulators as NumPy's pairwise leaf
    // Two lanes per 128-value leaf: lane h = 0 / 1 keeps NumPy's accumulators r0-r3 / r4-r7 (columns
    // 4h..4h+3 of each 8-value step, 16 steps of one row segment, 8-aligned because x0 is a multiple of
    // s/2 >= 8), so ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)) is one shuffle — the leaf order exactly.
    // Task u = 2 t + h for leaf t; every lane of the block runs the same number of rounds (shuffles).
    auto half_leaf = [&](int u, int& l, int& k, int& leaf, bool& live) -> T {
      const int t = u >> 1, h = u & 1;
      l = 0; k = 0; leaf = 0; live = false;
      if (t >= plan.nleaves) return T(0);
      l = plan.nlev - 1;
      while (lv[l].leaf0 < 0 || t < lv[l].leaf0) --l;
      const int s = lv[l].s, lsh = lv[l].lsh, msk = s - 1;
      const int lper = 2 * lsh - 7;  // log2 of the leaves per square
      k = (t - lv[l].leaf0) >> lper;
      leaf = (t - lv[l].leaf0) & ((1 << lper) - 1);
      live = k < lv[l].count;        // else an alignment gap before the next level
      if (!live) return T(0);
      int x0, y0;
      pre_square(lv[l], k, x0, y0);
      const T* b = img + y0 * ld + x0 + 4 * h;
      T r[4];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = (leaf << 7) + 8 * i;
        T w4[4];
        load4<T>(b + (q >> lsh) * ld + (q & msk), w4);
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = i == 0 ? w4[j] : r[j] + w4[j];
        if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // at most 8 steps of loads in flight
      }
      return (r[0] + r[1]) + (r[2] + r[3]);
    };
    if (PRE_DIAG(2)) {
    } else if constexpr (SK) {
      pre_leaves_sk<T>(img, ld, res, tid, lt_b, lt_m, plan.maxper);
      lds_barrier();
    } else if (!plan.tree_lds) {
      // a square's <= 32 leaves sit on 2 * per consecutive lanes of one wave (leaf0 is aligned to
      // per): the balanced tree over them (adjacent pairs first) by shuffles, the first lane stores
      // the mean
      for (int u0 = 0; u0 < 2 * plan.nleaves; u0 += kPreThreads) {
        int l, k, leaf;
        bool live;
        const int h = tid & 1;
        T v = half_leaf(u0 + tid, l, k, leaf, live);
        const int per = live ? (lv[l].s * lv[l].s) >> 7 : 0;
        {
          const T o = __shfl_down(v, 1, 64);
          if (h == 0) v = v + o;
        }
        for (int w = 1; w < plan.maxper; w <<= 1) {
          const T o = __shfl_down(v, 2 * w, 64);
          if (w < per && h == 0 && (leaf & (2 * w - 1)) == 0) v = v + o;
        }
        if (live && h == 0 && leaf == 0) res[lv[l].off + k] = pre_mean<T>(T(0) + v, 2 * lv[l].lsh);
      }
      lds_barrier();
    } else {
      for (int u0 = 0; u0 < 2 * plan.nleaves; u0 += kPreThreads) {
        int l, k, leaf;
        bool live;
        T v = half_leaf(u0 + tid, l, k, leaf, live);
        const T o = __shfl_down(v, 1, 64);
        if (live && (tid & 1) == 0) part[(u0 + tid) >> 1] = v + o;
      }
      lds_barrier();
    // balanced binary tree over each large square's leaves, adjacent pairs first (NumPy's split at
    // n/2 for n = 128 * 2^k is exactly this tree), one thread per square
    for (int a = plan.n_small + tid; a < plan.total; a += kPreThreads) {
      int l = 0;
      while (a >= lv[l].off + lv[l].count) ++l;
      const int per = (lv[l].s * lv[l].s) >> 7;
      T* pp = part + lv[l].leaf0 + (a - lv[l].off) * per;
      for (int w = 1; w < per; w <<= 1)
        for (int i = 0; i < per; i += 2 * w) pp[i] = pp[i] + pp[i + w];
      res[a] = pre_mean<T>(T(0) + pp[0], 2 * lv[l].lsh);
    }
    lds_barrier();
    }
    if (!PRE_DIAG(8)) pre_store(res, plan.total, out + e * out_stride, plan.nt, tid, kPreThreads);
    lds_barrier();
  }
}

// Skip runs of f32 1-D streams, wave-specialised: waves 0-1 load images PD ahead (float4 groups
// j = lane + 128 i) and scatter them into LDS, waves 2-3 store the previous image's averages, both
// before the image's first barrier; all four waves reduce.  On gfx9 the vector-memory counter is not
// ordered between loads and stores: in k_precomp the wait for the prefetched values (vmcnt(0)) also
// drained the previous image's stores every image.  Here the two roles run separate loops (the same
// barriers in the same order), so the loader waves' waits count loads only and the storer waves never
// wait on their stores.  Rows: 16-byte aligned (host), full groups read as float4 (the index clamped,
// no branch: a fixed number of loads per image, so waiting for image e leaves image e + grid in
// flight), a partial last group (d % 4) by four clamped dword loads.  Two barriers per image.  The LDS
// footprint (~30 KiB at n = 64, d = 1536) allows 5 workgroups per CU = 5 waves per SIMD: 96 VGPRs.
template <int KL, int PD, int LW = 2, bool CMP = false>
__global__ __launch_bounds__(kPreThreads) __attribute__((amdgpu_waves_per_eu(CMP ? 6 : 5))) void k_precomp_ws(
    const float* __restrict__ in, int64_t N, int64_t stride, int d, int n, PrePlan plan, float* __restrict__ out,
    int64_t out_stride, int ld, const uint16_t* __restrict__ glist) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ PreLevel lv[kPreMaxLevels];
  float* img = reinterpret_cast<float*>(smem);
  float* res = img + ((ld * n + 3) & ~3);  // no LDS tree on skip runs
  const int nres = CMP ? plan.znz : plan.total;  // CMP: the listed squares' averages only, by list position
  uint16_t* zl = reinterpret_cast<uint16_t*>(res + ((nres + 3) & ~3));
  const uint16_t* gmap = glist + pre_map_off(plan.znz);
  const int tid = threadIdx.x;
  constexpr int NL = 64 * LW;  // loader lanes (waves 0 .. LW - 1); the other waves store
  const int lt = tid < NL ? tid : tid - NL;
  const int lsh_n = plan.lsh_n;
  if (tid < plan.nlev) lv[tid] = plan.lv[tid];
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  pre_zero_setup<float>(img, res, zl, glist, plan.znz, nres, n, ld, tid);
  int lt_b = 0, lt_m = 0;
  pre_leaf_task(lv, plan, zl, ld, tid, lt_b, lt_m, CMP);
  const int64_t e0 = blockIdx.x, g = gridDim.x;
  if (e0 >= N) return;  // uniform over the workgroup
  auto reduce = [&] {
    if (!PRE_DIAG(1)) pre_small_levels<float, true, CMP>(lv, plan.nlev, img, ld, res, tid, zl);
    if (!PRE_DIAG(2)) pre_leaves_sk<float>(img, ld, res, tid, lt_b, lt_m, plan.maxper);
  };
  if (tid >= NL) {  // storer waves: no loads, so their stores are never waited on inside the loop
    int64_t prev = -1;
    PreMapRegs mr;
    mr.mis = -1;
    auto store = [&](int64_t e) {
      float* o = out + e * out_stride;
      if constexpr (CMP) {
        const int mis = (int)((reinterpret_cast<uintptr_t>(o) >> 2) & 3);
        if (mis != mr.mis) mr.load(gmap, plan.total, mis, lt, kPreThreads - NL);  // rows of another alignment
        pre_store_map(res, mr, plan.total, o, plan.nt, lt, kPreThreads - NL);
      } else {
        pre_store(res, plan.total, o, plan.nt, lt, kPreThreads - NL);
      }
    };
    for (int64_t e = e0; e < N; e += g) {
      if (prev >= 0 && !PRE_DIAG(8)) store(prev);
      lds_barrier();
      reduce();
      lds_barrier();
      prev = e;
    }
    if (!PRE_DIAG(8)) store(prev);
    return;
  }
  // loader waves
  const int G = (n * n) >> 2;
  const int nfull = d >> 2;  // full float4 groups (>= 1: host)
  uint32_t lut[KL];
  {
    const uint32_t* glut = n == 16 ? kPreLut16.v : (n == 32 ? kPreLut32.v : kPreLut64.v);
#pragma unroll
    for (int i = 0; i < KL; ++i) lut[i] = lt + NL * i < G ? glut[lt + NL * i] : 0u;
  }
  float pf[PD][KL][4];
  float tl[PD][4];  // the partial group nfull (d % 4 != 0): uniform scalar loads, substituted at the scatter
  auto fetch = [&](float (&p)[KL][4], float (&t)[4], int64_t e) {
    const float* src = in + e * stride;
    int nf = nfull, dd = d;
    asm volatile("" : "+s"(nf), "+s"(dd));
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const int j = min(lt + NL * i, nf - 1);
      const float4 q4 = *reinterpret_cast<const float4*>(src + 4 * j);
      p[i][0] = q4.x; p[i][1] = q4.y; p[i][2] = q4.z; p[i][3] = q4.w;
    }
    // the pf registers are written by these loads only (a VALU write here would make the compiler's wait
    // for one register set drain the other set's loads too)
#pragma unroll
    for (int m = 0; m < 4; ++m) t[m] = (dd & 3) ? src[min(4 * nf + m, dd - 1)] : 0.0f;
  };
  // plan.g2reg: a 2 x 2 grid square is a Hilbert group, so the loader averages it from the values it
  // scatters (NumPy's n < 8 sequential sum in C order, as pre_small<2>) and writes it after the barrier
  float g2v[KL];
  int g2k[KL];
  auto scatter = [&](const float (&p)[KL][4], const float (&tq)[4]) {
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const int j = lt + NL * i;
      int dz = d;
      asm volatile("" : "+s"(dz));
      g2k[i] = -1;
      if (j >= G || 4 * j >= dz) continue;  // padding stays +0.0 from the setup
      uint32_t ent = lut[i];
      asm volatile("" : "+v"(ent));
      const uint32_t off0 = ent & 0xFFFFu, code = ent >> 16;
      const uint32_t off = (off0 >> lsh_n) * ld + (off0 & (n - 1));
      const bool part = j == (dz >> 2);  // the partial group: its values from the scalar loads, zero-padded
      float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // values by position: (0,0) (0,1) (1,0) (1,1)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const uint32_t b = (code >> (2 * m)) & 3u;
        const float v = part ? (4 * j + m < dz ? tq[m] : 0.0f) : p[i][m];
        img[off + (b & 1u) + (b >> 1) * ld] = v;
#pragma unroll
        for (int t = 0; t < 4; ++t) c[t] = b == (uint32_t)t ? v : c[t];
      }
      if (plan.g2reg) {
        g2v[i] = pre_mean<float>(0.0f + ((((-0.0f + c[0]) + c[1]) + c[2]) + c[3]), 2);
        g2k[i] = (int)(((off0 >> lsh_n) >> 1) * (uint32_t)(n >> 1) + ((off0 & (n - 1)) >> 1));
      }
    }
  };
  auto g2_write = [&] {
    if (!plan.g2reg) return;
    const int o2 = lv[plan.g2lvl].off;
#pragma unroll
    for (int i = 0; i < KL; ++i)
      if (g2k[i] >= 0) res[o2 + g2k[i]] = g2v[i];
  };
  // every fetch issues its loads (past the last image the index is clamped to N - 1, loaded and never
  // used): no path without them, so the compiler's wait for set q counts the later sets' loads
#pragma unroll
  for (int q = 0; q < PD; ++q) fetch(pf[q], tl[q], min(e0 + q * g, N - 1));
  for (int64_t e = e0; e < N; e += PD * g) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      const int64_t ee = e + q * g;
      if (ee >= N) break;  // uniform
      scatter(pf[q], tl[q]);
      lds_barrier();
      fetch(pf[q], tl[q], min(ee + PD * g, N - 1));
      g2_write();
      reduce();
      lds_barrier();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Similarity (_compare_precomputed_levels / _calculate_precomputed_similarity) in the reference's
// float32 NumPy arithmetic.  Per vector and level (first m averages): mean, std (np.std: mean, then
// pairwise sum of squared deviations), mean of squares, and the normalised array (a - mean) / std.
// Per pair: corr = np.mean(qn * cn), mse = np.mean((q - c) ** 2), each a pairwise f32 sum divided as
// f32(f64(sum) / m).  Result types follow Python: the general branch yields float32, the constant
// branches (1.0 / 0.0 / 0.1) and the clamps Python floats; the weighted sum is float32 as soon as one
// float32 term enters it (a Python float operand is cast to float32), else float64.
// ------------------------------------------------------------------------------------------------
struct SimLevels {
  int nlev;
  int off_q[kPreMaxLevels], off_c[kPreMaxLevels], m[kPreMaxLevels];
  double w[kPreMaxLevels];  // normalised weights (Python floats)
};

template <class F>
__device__ __forceinline__ float np_mean32(const F& f, int m) {
  return (float)((double)np_sum<float>(f, m) / (double)m);
}

// stats [N, nlev, 3] = (mean, std, mean of squares); norm [N, T]: normalised averages (std != 0)
__global__ __launch_bounds__(256) void k_pre_stats(const float* __restrict__ A, int64_t N, int64_t stride, int nlev,
                                                   SimLevels L, int side, float* __restrict__ stats,
                                                   float* __restrict__ norm) {
  const int64_t total = N * nlev;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = t / nlev;
    const int l = (int)(t % nlev);
    const int m = L.m[l];
    const int off = side == 0 ? L.off_q[l] : L.off_c[l];
    const float* a = A + v * stride + off;
    float* st = stats + t * 3;
    if (m <= 0) {
      st[0] = st[1] = st[2] = 0.0f;
      continue;
    }
    const float mean = np_mean32([&](int k) { return a[k]; }, m);
    const float var = np_mean32([&](int k) { const float dd = a[k] - mean; return dd * dd; }, m);
    const float sd = sqrtf(var);
    const float msq = np_mean32([&](int k) { return a[k] * a[k]; }, m);
    st[0] = mean;
    st[1] = sd;
    st[2] = msq;
    float* o = norm + v * stride + off;
    if (sd != 0.0f)
      for (int k = 0; k < m; ++k) o[k] = (a[k] - mean) / sd;
  }
}

// out_overall [Q, N] f64 value, out_type [Q, N] (0: float32, 1: Python float), out_levels
// [Q, N, nlev] f64 (may be null)
__global__ __launch_bounds__(256) void k_pre_pairs(const float* __restrict__ Qa, const float* __restrict__ Qn,
                                                   const float* __restrict__ Qs, int Qc, int64_t qstride,
                                                   const float* __restrict__ Ca, const float* __restrict__ Cn,
                                                   const float* __restrict__ Cs, int64_t N, int64_t cstride,
                                                   SimLevels L, double* __restrict__ out_overall,
                                                   uint8_t* __restrict__ out_type, double* __restrict__ out_levels) {
  const int64_t total = (int64_t)Qc * N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t qi = t / N, ci = t % N;
    double acc = 0.0;
    int acc_t = -1;  // -1: int 0 (nothing added yet), 0: float32, 1: Python float
    for (int l = 0; l < L.nlev; ++l) {
      const int m = L.m[l];
      const float* qs = Qs + (qi * L.nlev + l) * 3;
      const float* cs = Cs + (ci * L.nlev + l) * 3;
      double sim;
      int st;  // type of the level similarity
      if (m <= 0) {
        sim = 0.0;
        st = 1;
      } else if (qs[1] == 0.0f && cs[1] == 0.0f) {
        sim = fabsf(qs[0] - cs[0]) < 1e-6f ? 1.0 : 0.0;  // Python float compared in float32 (NEP 50)
        st = 1;
      } else if (qs[1] == 0.0f || cs[1] == 0.0f) {
        sim = 0.1;
        st = 1;
      } else {
        const float* qa = Qa + qi * qstride + L.off_q[l];
        const float* ca = Ca + ci * cstride + L.off_c[l];
        const float* qn = Qn + qi * qstride + L.off_q[l];
        const float* cn = Cn + ci * cstride + L.off_c[l];
        const float corr = np_mean32([&](int k) { return qn[k] * cn[k]; }, m);
        const float corr_sim = (corr + 1.0f) / 2.0f;
        const float mse = np_mean32([&](int k) { const float dd = qa[k] - ca[k]; return dd * dd; }, m);
        const float maxm = qs[2] + cs[2];
        float ds;
        if (maxm > 0.0f) {
          ds = 1.0f - mse / maxm;
          ds = ds > 0.0f ? ds : 0.0f;
        } else {
          ds = 1.0f;
        }
        const float comb = 0.7f * corr_sim + 0.3f * ds;
        if (comb < 1.0f && comb > 0.0f) {
          sim = comb;
          st = 0;
        } else {
          sim = comb < 1.0f ? 0.0 : 1.0;
          st = 1;
        }
      }
      if (out_levels) out_levels[t * L.nlev + l] = sim;
      // term = sim * w (float32 if sim is float32), then acc + term with Python/NEP 50 typing
      const double term = st == 0 ? (double)((float)sim * (float)L.w[l]) : sim * L.w[l];
      if (acc_t < 0) {
        acc = term;
        acc_t = st;
      } else if (acc_t == 1 && st == 1) {
        acc = acc + term;
      } else {
        acc = (double)((float)acc + (float)term);
        acc_t = 0;
      }
    }
    if (acc_t < 0) acc_t = 1;
    double v = acc < 1.0 ? acc : 1.0;
    if (!(acc < 1.0)) acc_t = 1;
    if (!(v > 0.0)) { v = 0.0; acc_t = 1; }
    out_overall[t] = v;
    out_type[t] = (uint8_t)acc_t;
  }
}

// Legacy compare_indices_at_level of the pre-computed engine (:468-496): np.std branches, np.allclose
// for two constant vectors, else (np.corrcoef(q, c)[0, 1] + 1) / 2 (0.0 when NaN).  corrcoef goes
// through np.cov's BLAS dot, whose summation order is not NumPy's pairwise order: the centred dot
// products here are sequential fma chains (agreement ~1e-15 relative, not bit-exact).
__global__ __launch_bounds__(256) void k_pearson(const double* __restrict__ q, const double* __restrict__ C, int64_t N,
                                                 int m, double* __restrict__ out) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    const double* x = C + c * m;
    const double qm = np_sum<double>([=](int k) { return q[k]; }, m) / (double)m;
    const double cm = np_sum<double>([=](int k) { return x[k]; }, m) / (double)m;
    const double qs = sqrt(np_sum<double>([=](int k) { const double d = q[k] - qm; return d * d; }, m) / (double)m);
    const double cs = sqrt(np_sum<double>([=](int k) { const double d = x[k] - cm; return d * d; }, m) / (double)m);
    double r;
    if (qs == 0.0 && cs == 0.0) {
      bool close = true;  // np.allclose(q, c): |q - c| <= 1e-8 + 1e-5 |c|
      for (int k = 0; k < m; ++k) close &= fabs(q[k] - x[k]) <= 1e-8 + 1e-5 * fabs(x[k]);
      r = close ? 1.0 : 0.0;
    } else if (qs == 0.0 || cs == 0.0) {
      r = 0.1;
    } else {
      double c00 = 0.0, c11 = 0.0, c01 = 0.0;
      for (int k = 0; k < m; ++k) {
        const double a = q[k] - qm, b = x[k] - cm;
        c00 = fma(a, a, c00);
        c11 = fma(b, b, c11);
        c01 = fma(a, b, c01);
      }
      const double f = 1.0 / (double)(m - 1);
      double corr = (c01 * f) / sqrt(c00 * f) / sqrt(c11 * f);
      corr = corr > 1.0 ? 1.0 : (corr < -1.0 ? -1.0 : corr);
      r = corr == corr ? (corr + 1.0) / 2.0 : 0.0;
    }
    out[c] = r;
  }
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_precomputed_layout(int n, int max_levels, int min_square_size, int32_t* levels_out, int max_out) {
  if (n <= 0 || !is_pow2(n) || max_levels <= 0 || min_square_size <= 0)
    return fail(HQ_E_INVALID, "bad layout request n=%d", n);
  PrePlan p;
  if (pre_plan(n, max_levels, min_square_size, p) != HQ_OK) return fail(HQ_E_UNSUPPORTED, "layout n=%d", n);
  for (int i = 0; i < p.nlev && i < max_out; ++i) {
    levels_out[4 * i + 0] = p.lv[i].g;
    levels_out[4 * i + 1] = p.lv[i].s;
    levels_out[4 * i + 2] = p.lv[i].count;
    levels_out[4 * i + 3] = p.lv[i].off;
  }
  return p.nlev;
}

int hq_precomputed_index(int dtype, int kind, const void* in, int64_t N, int64_t in_stride, int d, int n,
                         int max_levels, int min_square_size, float* out, int64_t out_stride, hq_stream_t stream) {
  if (N < 0 || n <= 0 || in_stride < 0) return fail(HQ_E_INVALID, "bad shape");
  if (!is_pow2(n)) return fail(HQ_E_NOT_POW2, "Dimension must be a power of 2, got %d", n);
  if (n > 128) return fail(HQ_E_UNSUPPORTED, "pre-computed index of a %dx%d image (n <= 128)", n, n);
  if (kind != 0 && kind != 1) return fail(HQ_E_INVALID, "kind %d", kind);
  if (kind == 1 && (d < 0 || d > n * n)) return fail(HQ_E_TOO_MANY, "%d values for a %dx%d image", d, n, n);
  if (N == 0) return HQ_OK;
  if (!in || !out) return fail(HQ_E_INVALID, "null buffer");
  PrePlan p;
  if (max_levels <= 0 || min_square_size <= 0) return fail(HQ_E_INVALID, "max_levels / min_square_size");
  if (pre_plan(n, max_levels, min_square_size, p) != HQ_OK)
    return fail(HQ_E_UNSUPPORTED, "layout n=%d max_levels=%d min_square_size=%d (power-of-two squares, <= 8 levels)",
                n, max_levels, min_square_size);
  if (out_stride < p.total) return fail(HQ_E_INVALID, "out_stride %lld < %d averages", (long long)out_stride, p.total);
  p.nt = opt(OPT_PRECOMP_NT, p.nt) != 0;
  p.leaf_rot = opt(OPT_PRECOMP_LEAF_ROT, 1) != 0;  // A/B
  if (opt_on(OPT_PRECOMP_TREE_LDS)) p.tree_lds = 1;  // A/B: combine leaves through LDS
#ifdef HQ_DIAG  // phase-skipping diagnostics (wrong averages): A/B builds only (make DIAG=1)
  p.diag = (int)opt(OPT_PRECOMP_DIAG, p.diag);
#endif
  const int esz = dtype == HQ_F64 ? 8 : 4;
  const int pad = (int)opt(OPT_PRECOMP_PAD, 4);
  if (pad < 0 || (pad & 3)) return fail(HQ_E_INVALID, "option precomp_pad must be a multiple of 4");
  const int ld = n + pad;
  const int use_lut = kind == 1 && n >= 16 && n <= 64;  // compile-time group LUT exists for this n
  // zero-padding skip (pre_zero_plan): 1-D streams with padding, leaves combined in registers;
  // A/B: option precomp_skip = 0 computes every square
  const bool skip = use_lut && !p.tree_lds && opt(OPT_PRECOMP_SKIP, 1) != 0 && pre_zero_plan(n, d, p);
  // skip runs of f32 streams take the wave-specialised kernel when the row bases are 16-byte aligned and
  // the groups below d fit 128 loader lanes x 4 (A/B: option precomp_ws = 0 keeps k_precomp; 2
  // prefetches two images ahead: 4.36 vs 4.23 ms for one, the compiler's waits still drain both sets)
  const int ngroups = (d + 3) / 4;
  const int64_t ws = opt(OPT_PRECOMP_WS, 1);
  const bool use_ws = dtype == HQ_F32 && skip && ws != 0 && d >= 4 && ngroups <= 128 * 4 &&
                      (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (in_stride & 3) == 0;
  // option precomp_g2reg = 1: the 2 x 2 grid squares from the loader's registers (A/B: 4.12-4.15 vs
  // 3.96-4.01 ms without: the loaders' scatter phase is the longer side of the first phase)
  if (use_ws && p.g2lvl >= 0 && opt(OPT_PRECOMP_G2REG, 0) != 0) {
    p.g2reg = 1;  // its 2 x 2 grid squares come from the loader's registers: re-list without them
    pre_zero_plan(n, d, p);
  }
  // skip runs: the square lists, built on the host once per configuration (A/B: option
  // precomp_order = 0 keeps them in square order instead of the LDS bank order)
  const uint16_t* glist = nullptr;
  if (skip) {
    int err = HQ_OK;
    glist = pre_zero_lists(n, d, ld, esz, max_levels, min_square_size, (int)opt(OPT_PRECOMP_ORDER, 1), p,
                           (hipStream_t)stream, err);
    if (!glist) return fail(err, "pre-computed index: zero-padding lists (n=%d d=%d)", n, d);
  }
  // option precomp_compact = 1: the wave-specialised skip runs keep only the listed squares' averages in LDS
  // (30.2 -> 23.5 KB at n = 64, d = 1536: six workgroups per CU instead of five).  A/B on one box (ms per
  // 1M x 1536): 4.114 / 4.117 vs 4.085 / 4.088 without — more resident images do not help (the mixed
  // read/write HBM stream bounds the kernel), so it is off by default
  const bool cmp = skip && !p.g2reg && p.total <= 128 * 4 * kPreStoreG && opt(OPT_PRECOMP_COMPACT, 0) != 0;
  const size_t lds_ws = (size_t)esz * ((size_t)((ld * n + 3) & ~3)) + 4 * (size_t)(((cmp ? p.znz : p.total) + 3) & ~3) +
                        (skip ? 2 * (size_t)p.znz : 0);
  const size_t lds = (size_t)esz * ((size_t)((ld * n + 3) & ~3) + (p.tree_lds ? p.nleaves_al : 0)) + 4 * (size_t)((p.total + 3) & ~3) +
                     (skip ? 2 * (size_t)p.znz : 0);
  if (lds > 160 * 1024) return fail(HQ_E_UNSUPPORTED, "pre-computed index n=%d dtype %d needs %zu B of LDS", n, dtype, lds);
  hipStream_t s = (hipStream_t)stream;
  // skip runs: a workgroup loops over many images (the list setup is amortised) and prefetches the
  // next image into registers (A/B, M emb/s at d = 1536: grid 262144 / 16384 / 8192 without prefetch
  // 110 / 169 / 157, with it 125 / 192 / 195; no skip 142)
  const int64_t gcap = opt(OPT_PRECOMP_GRID, skip ? 8192 : 65536 * 4);  // A/B: workgroups (each loops over images)
  const int64_t grid64 = N < gcap ? N : (gcap > 0 ? gcap : 1);
  const int pf = (int)opt(OPT_PRECOMP_PF, skip ? 1 : 0);  // A/B: 1 = prefetch the next image into registers
  if (dtype == HQ_F32) {
    // groups of 4 values a thread scatters: a skip run touches only groups below d
    const bool kg2 = skip && (d + 3) / 4 <= 2 * kPreThreads;
    if (use_ws) {
      const int kl = ngroups <= 128 * 2 ? 2 : (ngroups <= 128 * 3 ? 3 : 4);
      auto wk = ws == 1 ? (kl == 2 ? k_precomp_ws<2, 1> : (kl == 3 ? k_precomp_ws<3, 1> : k_precomp_ws<4, 1>))
                        : (kl == 2 ? k_precomp_ws<2, 2> : (kl == 3 ? k_precomp_ws<3, 2> : k_precomp_ws<4, 2>));
      if (cmp && ws == 1)
        wk = kl == 2 ? k_precomp_ws<2, 1, 2, true> : (kl == 3 ? k_precomp_ws<3, 1, 2, true> : k_precomp_ws<4, 1, 2, true>);
      // ws = 3: three loader waves and one storer (groups per loader lane ceil(ngroups / 192))
      if (ws == 3) {
        const int k3 = ngroups <= 192 * 2 ? 2 : 3;
        wk = k3 == 2 ? k_precomp_ws<2, 1, 3> : k_precomp_ws<3, 1, 3>;
      }
      // more workgroups than the 1,280 resident ones desynchronise the phases of a CU's workgroups
      // (A/B, ms at 1M x 1536: grid 1280 / 5120 / 8192 / 20480 / 65536 -> 4.50 / 4.05 / 3.98 / 3.91 /
      // 4.01); the averages are written once but plain stores measured ~1% faster than non-temporal
      const int64_t wcap = opt(OPT_PRECOMP_GRID, 20480);
      const int64_t wgrid = N < wcap ? N : (wcap > 0 ? wcap : 1);
      p.nt = opt(OPT_PRECOMP_NT, 0) != 0;
      const size_t lw = cmp && ws == 1 ? lds_ws : lds;
      HQ_CHECK_HIP(hipFuncSetAttribute((const void*)wk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lw));
      hipLaunchKernelGGL(wk, dim3((unsigned)wgrid), dim3(kPreThreads), lw, s, (const float*)in, N, in_stride, d, n,
                         p, out, out_stride, ld, glist);
      HQ_CHECK_LAUNCH();
      return HQ_OK;
    }
    auto kern = skip ? (kg2 ? (pf ? k_precomp<float, 1, true, 2> : k_precomp<float, 0, true, 2>)
                            : (pf ? k_precomp<float, 1, true, 4> : k_precomp<float, 0, true, 4>))
                     : (pf ? k_precomp<float, 1, false, 4> : k_precomp<float, 0, false, 4>);
    HQ_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)grid64), dim3(kPreThreads), lds, s, (const float*)in, kind, N,
                       in_stride, d, n, p, out, out_stride, use_lut, ld, glist);
  } else if (dtype == HQ_F64) {
    auto kern = skip ? k_precomp<double, 0, true, 4> : k_precomp<double, 0, false, 4>;
    HQ_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)grid64), dim3(kPreThreads), lds, s, (const double*)in, kind,
                       N, in_stride, d, n, p, out, out_stride, use_lut, ld, glist);
  } else {
    return fail(HQ_E_UNSUPPORTED, "pre-computed index dtype %d (f32/f64)", dtype);
  }
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_pearson_f64(const double* q, const double* C, int64_t N, int m, double* out, hq_stream_t stream) {
  if (N < 0 || m <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (N == 0) return HQ_OK;
  if (!q || !C || !out) return fail(HQ_E_INVALID, "null buffer");
  int64_t blocks = (N + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_pearson, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, q, C, N, m, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_precomputed_stats(const float* avgs, int64_t N, int64_t stride, int nlev, const int32_t* offsets,
                         const int32_t* counts, float* stats, float* norm, hq_stream_t stream) {
  if (N < 0 || nlev <= 0 || nlev > kPreMaxLevels || !offsets || !counts) return fail(HQ_E_INVALID, "bad levels");
  if (N == 0) return HQ_OK;
  if (!avgs || !stats || !norm) return fail(HQ_E_INVALID, "null buffer");
  SimLevels L{};
  L.nlev = nlev;
  for (int l = 0; l < nlev; ++l) { L.off_q[l] = offsets[l]; L.off_c[l] = offsets[l]; L.m[l] = counts[l]; }
  int64_t blocks = (N * nlev + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_pre_stats, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, avgs, N, stride, nlev, L,
                     0, stats, norm);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_precomputed_similarity(const float* q_avgs, const float* q_norm, const float* q_stats, int Q, int64_t q_stride,
                              const float* c_avgs, const float* c_norm, const float* c_stats, int64_t N,
                              int64_t c_stride, int nlev, const int32_t* q_offsets, const int32_t* c_offsets,
                              const int32_t* counts, const double* weights, double* out_overall, uint8_t* out_type,
                              double* out_levels, hq_stream_t stream) {
  if (Q < 0 || N < 0 || nlev <= 0 || nlev > kPreMaxLevels) return fail(HQ_E_INVALID, "bad shape");
  if (!q_offsets || !c_offsets || !counts || !weights) return fail(HQ_E_INVALID, "null level table");
  if (Q == 0 || N == 0) return HQ_OK;
  if (!q_avgs || !q_norm || !q_stats || !c_avgs || !c_norm || !c_stats || !out_overall || !out_type)
    return fail(HQ_E_INVALID, "null buffer");
  SimLevels L{};
  L.nlev = nlev;
  for (int l = 0; l < nlev; ++l) {
    L.off_q[l] = q_offsets[l];
    L.off_c[l] = c_offsets[l];
    L.m[l] = counts[l];
    L.w[l] = weights[l];
  }
  int64_t blocks = ((int64_t)Q * N + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_pre_pairs, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, q_avgs, q_norm, q_stats,
                     Q, q_stride, c_avgs, c_norm, c_stats, N, c_stride, L, out_overall, out_type, out_levels);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // extern "C"
