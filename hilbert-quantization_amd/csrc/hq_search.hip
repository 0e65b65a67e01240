// hq_search.hip — hierarchical-index similarity scan.
//
// Reference: core/search_engine.py:42-388 (ProgressiveSimilaritySearchEngine), core/video_search.py:
// 215-264,1316-1328 (level-0 scan over stored frames), rag/search/engine.py:622-660,1025-1051 (cosine).
//
// compare_indices_at_level (search_engine.py:111-189) for one level segment of length m is
//   both std 0 -> |mean_q - mean_c| < 1e-6 ? 1 : 0;  one std 0 -> 0.1;  otherwise
//   corr = mean(zq*zc), sim = (corr+1)/2, dsim = max(0, 1 - mse/maxmse), clamp(0.7 sim + 0.3 dsim)
// with zq = (q - mean_q)/std_q.  Everything except G = sum_j zq_j zc_j is a per-vector statistic, so
// the scan is a segmented f64 GEMM (v_mfma_f64_16x16x4f64) plus an epilogue:
//   corr = G/m;  sum q*c = std_q std_c G + m mean_q mean_c;
//   1 - mse/maxmse = 2 (sum q*c) / (m (msq_q + msq_c))      (msq = mean of squares)
// Zero-variance branches are decided by std values computed in NumPy's pairwise order
// (k_seg_prepare), so the exact-constant outcomes (0, 0.1, 1) are bit-identical to the reference.
//
// Index vectors are stored "segment padded": each level segment starts at a multiple of 4 f64 and
// is zero-filled to a multiple of 4 (Lp columns), so every MFMA k-step lies inside one segment.
#include <type_traits>
#include "hq_common.h"

#include <math.h>

namespace hq {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// Bounds guard of the DIAG build (make DIAG=1): HQ_GUARD(p, base, lim) checks that the element offset
// p - base lies in [0, lim); a violation is counted (hq_diag_violations, with the source line of the
// first one) and the pointer is clamped, so a faulty corpus-row index shows up as a count, never as a
// GPU fault.  The default build compiles the guard away.
#ifdef HQ_DIAG
__device__ unsigned long long g_diag_count;
__device__ int g_diag_line;
__device__ __noinline__ int64_t diag_bound(int64_t off, int64_t lim, int line) {
  if (off >= 0 && off < lim) return off;
  if (atomicAdd(&g_diag_count, 1ull) == 0ull) atomicExch(&g_diag_line, line);
  return off < 0 ? 0 : (lim > 0 ? lim - 1 : 0);
}
#define HQ_GUARD(p, base, lim) ((p) = (base) + diag_bound((int64_t)((p) - (base)), (int64_t)(lim), __LINE__))
#else
#define HQ_GUARD(p, base, lim) ((void)0)
#endif

// ------------------------------------------------------------------------------------------------
// segment layout
// ------------------------------------------------------------------------------------------------
struct SegInfo {
  int nseg;
  int L, Lp;
  int src[kMaxSeg];   // start in the raw index vector
  int len[kMaxSeg];   // segment length m
  int poff[kMaxSeg];  // start in the padded layout (multiple of 4)
  int plen[kMaxSeg];  // padded length (multiple of 4)
  double inv_m[kMaxSeg];
  double w[kMaxSeg];  // 1/(l+1) (search_engine.py:205)
  double wsum;
};

static void seg_info(int L, SegInfo& s) {
  SegTable t;
  parse_structure(L, L, t);
  s.nseg = t.nseg;
  s.L = L;
  int off = 0;
  s.wsum = 0.0;
  for (int i = 0; i < t.nseg; ++i) {
    s.src[i] = t.start[i];
    s.len[i] = t.end[i] - t.start[i];
    s.poff[i] = off;
    s.plen[i] = (s.len[i] + 3) & ~3;
    off += s.plen[i];
    s.inv_m[i] = 1.0 / (double)s.len[i];
    s.w[i] = 1.0 / (double)(i + 1);
    s.wsum += s.w[i];
  }
  s.Lp = off;
}

// ------------------------------------------------------------------------------------------------
// per-segment statistics + normalised vectors (reference np.mean/np.std order)
//
// stats[row][seg] = (mean, std, msq, aux): the model the APPROXIMATE scans evaluate (Z = normalised
// values, score from G = sum zq zc, corr = G / m, sum q c = std_q std_c G + m mean_q mean_c).
// f64 sources: NumPy f64 statistics, z = (x - mean) / std, aux = 0.
// f32 sources (src_f32): the reference runs np.std / np.mean and the normalisation in float32
// (NumPy keeps the array dtype), so z = f32((x - mean32) / std32), std = std32 (float32 pairwise
// order) — the reference's own normalised values.  Their sum is m (mean64 - mean32) / std32, not 0,
// so the identity for sum q c needs the exact (f64) means: mean = mean64 (the dropped product of the
// two mean errors is ~1e-14 relative).  A segment whose float32 std is 0 (the reference's constant
// branch) stores the float32 mean (compared in float32 there) and std 0.  aux bits (as a double):
//   kAuxF32    float32 source: the exact path recomputes this vector's statistics, z and (when the
//              other side is float32 too) the whole score in float32
//   kAuxUnsafe mean of squares outside [2^-100, 2^100]: float32 squares under/overflow in the
//              reference, which the model does not follow; callers score such vectors on the dense
//              exact path
// ------------------------------------------------------------------------------------------------
constexpr int kAuxF32 = 1, kAuxUnsafe = 2;

__device__ __forceinline__ int aux_bits(const double* st) { return (int)st[3]; }

// one (row, segment): x = the row's raw values (global memory or an LDS copy of the row)
__device__ __forceinline__ void seg_prepare_one(const double* xrow, int64_t row, int s, const SegInfo& si,
                                                int all_f32, const uint8_t* __restrict__ row_f32,
                                                double* __restrict__ Z, double* __restrict__ stats) {
  const double* x = xrow + si.src[s];
  const int m = si.len[s];
  auto fx = [=](int k) -> double { return x[k]; };
  const double mean = np_sum<double>(fx, m) / (double)m;            // np.mean
  auto fd = [=](int k) -> double { double d = x[k] - mean; return d * d; };
  const double sd = sqrt(np_sum<double>(fd, m) / (double)m);        // np.std (_methods._var)
  auto fs = [=](int k) -> double { return x[k] * x[k]; };
  const double msq = np_sum<double>(fs, m) / (double)m;             // np.mean(q ** 2)
  double* z = Z + row * si.Lp + si.poff[s];
  double* st = stats + (row * si.nseg + s) * 4;
  if (row_f32 ? row_f32[row] != 0 : all_f32 != 0) {
    // _methods._var on float32: f32 pairwise sum, divide, x - mean, x * x, f32 pairwise sum, divide,
    // sqrt (np.mean = f32(f64(sum) / m) = the f32 division: the double rounding is innocuous)
    auto gx = [=](int k) -> float { return (float)x[k]; };
    const float mean32 = np_sum<float>(gx, m) / (float)m;
    auto gd = [=](int k) -> float { float d = (float)x[k] - mean32; return d * d; };
    const float sd32 = sqrtf(np_sum<float>(gd, m) / (float)m);
    int aux = kAuxF32;
    if (!(msq >= 0x1p-100 && msq <= 0x1p100)) aux |= kAuxUnsafe;
    if (sd32 == 0.0f) {
      for (int i = 0; i < si.plen[s]; ++i) z[i] = 0.0;
      st[0] = (double)mean32;
      st[1] = 0.0;
    } else {
      for (int i = 0; i < m; ++i) z[i] = (double)(((float)x[i] - mean32) / sd32);  // (q - mean(q)) / std
      for (int i = m; i < si.plen[s]; ++i) z[i] = 0.0;
      st[0] = mean;
      st[1] = (double)sd32;
    }
    st[2] = msq;
    st[3] = (double)aux;
    return;
  }
  if (sd == 0.0) {
    for (int i = 0; i < si.plen[s]; ++i) z[i] = 0.0;
  } else {
    for (int i = 0; i < m; ++i) z[i] = (x[i] - mean) / sd;          // (q - mean(q)) / std (:150-151)
    for (int i = m; i < si.plen[s]; ++i) z[i] = 0.0;
  }
  st[0] = mean;
  st[1] = sd;
  st[2] = msq;
  st[3] = 0.0;
}

__global__ __launch_bounds__(256) void k_seg_prepare(const double* __restrict__ idx, int64_t N, SegInfo si,
                                                     int all_f32, const uint8_t* __restrict__ row_f32,
                                                     double* __restrict__ Z, double* __restrict__ stats) {
  const int64_t total = N * si.nseg;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / si.nseg;
    seg_prepare_one(idx + row * si.L, row, (int)(t % si.nseg), si, all_f32, row_f32, Z, stats);
  }
}

// Small batches (query preparation: 1,000 rows x 5 segments is only ~20 workgroups of the kernel
// above, each thread walking three dependent chains of global loads, ~18 us): one wave per row copies
// the row to LDS with one coalesced load, then one lane per segment runs the same arithmetic on the
// LDS copy (bit-identical results).
__global__ __launch_bounds__(64) void k_seg_prepare_lds(const double* __restrict__ idx, int64_t N, SegInfo si,
                                                        int all_f32, const uint8_t* __restrict__ row_f32,
                                                        double* __restrict__ Z, double* __restrict__ stats) {
  extern __shared__ double xs[];  // L values
  const int lane = threadIdx.x;
  for (int64_t row = blockIdx.x; row < N; row += gridDim.x) {
    for (int i = lane; i < si.L; i += 64) xs[i] = idx[row * si.L + i];
    __syncthreads();
    for (int s = lane; s < si.nseg; s += 64) seg_prepare_one(xs, row, s, si, all_f32, row_f32, Z, stats);
    __syncthreads();
  }
}

// constant branches of compare_indices_at_level (search_engine.py:141-148); both32: both arrays are
// float32, so the mean difference and the 1e-6 literal are float32 (NEP 50)
__device__ __forceinline__ double const0(bool zq, bool zc, double qm, double cm, bool both32 = false) {
  if (zq && zc) {
    if (both32) return fabsf((float)qm - (float)cm) < 1e-6f ? 1.0 : 0.0;
    return fabs(qm - cm) < 1e-6 ? 1.0 : 0.0;
  }
  return 0.1;
}

// score of one level from the contraction G and the two vectors' segment statistics
__device__ __forceinline__ double level_sim(double G, double qm, double qs, double qq, double cm, double cs,
                                            double cq, double m, double inv_m, bool both32 = false) {
  const bool fq = qs == 0.0, fc = cs == 0.0;
  if (fq || fc) return const0(fq, fc, qm, cm, both32);
  const double corr = G * inv_m;
  const double sim = (corr + 1.0) * 0.5;
  const double t1 = (qs * cs) * G;
  const double t2 = (qm * cm) * m;
  const double dot = t1 + t2;                 // sum q*c
  const double maxmse = qq + cq;              // > 0 here: both segments have a non-zero value
  double dsim = (2.0 * inv_m) * dot / maxmse; // 1 - mse / maxmse
  dsim = dsim > 0.0 ? dsim : 0.0;
  double comb = 0.7 * sim + 0.3 * dsim;
  comb = comb < 1.0 ? comb : 1.0;
  return comb > 0.0 ? comb : 0.0;
}

// ------------------------------------------------------------------------------------------------
// EXACT scores: compare_indices_at_level (search_engine.py:111-189) in the reference's operation
// order — products and squared differences summed in NumPy's pairwise order, then the same Python
// float expression.  Used for dense scores, re-scoring and the final re-rank of the MFMA scan's
// candidate lists, so rankings (including noise-level ties) match the reference bit for bit.
// ------------------------------------------------------------------------------------------------
struct VecSet {
  const double* raw;  // N x L  (original index vectors)
  const double* Z;    // N x Lp (segment-padded normalised vectors)
  const double* S;    // N x nseg x 4 (mean, std, mean of squares, 0)
};

// One side of a level comparison: the raw segment, its normalised copy (f64 sides) and statistics in
// the side's own dtype.  f32 sides recompute np.mean / np.std / np.mean(x ** 2) in float32 NumPy order.
struct Side {
  const double* x;  // raw values (f32 sources hold float32 values)
  const double* z;  // (x - mean) / std in f64 (f64 sides); null: computed on the fly
  double mean, sd, msq;
  bool f32;
};

template <bool SM = false>
__device__ __forceinline__ Side make_side(const double* x, const double* z, const double* st, int m, bool f32) {
  Side r;
  r.x = x;
  r.z = z;
  r.f32 = f32;
  if (f32) {
    auto gx = [=](int k) -> float { return (float)x[k]; };
    const float mean = np_sum<float, SM>(gx, m) / (float)m;
    auto gd = [=](int k) -> float { const float d = (float)x[k] - mean; return d * d; };
    const float sd = sqrtf(np_sum<float, SM>(gd, m) / (float)m);
    auto gs = [=](int k) -> float { const float v = (float)x[k]; return v * v; };
    r.mean = mean;
    r.sd = sd;
    r.msq = np_sum<float, SM>(gs, m) / (float)m;
  } else if (st) {
    r.mean = st[0];
    r.sd = st[1];
    r.msq = st[2];
  } else {
    auto fx = [=](int k) -> double { return x[k]; };
    r.mean = np_sum<double, SM>(fx, m) / (double)m;
    const double mu = r.mean;
    auto fd = [=](int k) -> double { const double d = x[k] - mu; return d * d; };
    r.sd = sqrt(np_sum<double, SM>(fd, m) / (double)m);
    auto fs = [=](int k) -> double { return x[k] * x[k]; };
    r.msq = np_sum<double, SM>(fs, m) / (double)m;
  }
  return r;
}

// element k of the side's normalised array ((q - np.mean(q)) / q_std in the side's dtype)
__device__ __forceinline__ double side_z(const Side& s, int k) {
  if (s.f32) return (double)(((float)s.x[k] - (float)s.mean) / (float)s.sd);
  if (s.z) return s.z[k];
  return (s.x[k] - s.mean) / s.sd;
}

// compare_indices_at_level (search_engine.py:111-189) for one segment in the reference's operation
// order and dtype.  *np32 = 1 when the result is a numpy float32 (both sides f32, general branch,
// not clamped), else it is a Python float: the type decides the overall weighted sum's arithmetic.
// F2: the correlation's products and the squared differences summed in one pass (Sum2: each sum in its
// own pairwise order, bit-identical; every element read once, 16 more VGPRs — the long-list re-rank, whose
// per-thread row reads are request-bound, uses it)
template <bool SM = false, bool F2 = false>
__device__ double exact_level_sides(const Side& q, const Side& c, int m, int* np32) {
  *np32 = 0;
  const bool both32 = q.f32 && c.f32;
  if (q.sd == 0.0 || c.sd == 0.0) return const0(q.sd == 0.0, c.sd == 0.0, q.mean, c.mean, both32);  // :141-148
  if (both32) {
    // float32 throughout: np.mean = f32(f64(f32 pairwise sum) / m) = f32 division (exact double
    // rounding); Python float literals are cast to float32 (NEP 50); no FMA contraction
    float corr, mse;
    if constexpr (F2) {
      auto f2 = [&](int k) -> Sum2<float> {
        const float d = (float)q.x[k] - (float)c.x[k];
        return Sum2<float>((float)side_z(q, k) * (float)side_z(c, k), d * d);
      };
      const Sum2<float> s2 = np_sum<Sum2<float>, SM>(f2, m);
      corr = s2.a / (float)m;
      mse = s2.b / (float)m;
    } else {
      auto fp = [&](int k) -> float { return (float)side_z(q, k) * (float)side_z(c, k); };
      corr = np_sum<float, SM>(fp, m) / (float)m;                                   // :154
      auto fd = [&](int k) -> float { const float d = (float)q.x[k] - (float)c.x[k]; return d * d; };
      mse = np_sum<float, SM>(fd, m) / (float)m;                                    // :161
    }
    const float sim = (corr + 1.0f) / 2.0f;                                        // :158
    const float maxmse = (float)q.msq + (float)c.msq;                              // :162
    float ds = 1.0f;
    if (maxmse > 0.0f) {
      ds = 1.0f - mse / maxmse;
      ds = ds > 0.0f ? ds : 0.0f;
    }
    const float comb = 0.7f * sim + 0.3f * ds;                                     // :171
    if (comb < 1.0f && comb > 0.0f) {
      *np32 = 1;
      return comb;
    }
    return comb < 1.0f ? 0.0 : 1.0;                                                // :174 (Python floats)
  }
  double corr, mse;
  if constexpr (F2) {
    auto f2 = [&](int k) -> Sum2<double> {
      const double d = q.x[k] - c.x[k];
      return Sum2<double>(side_z(q, k) * side_z(c, k), d * d);
    };
    const Sum2<double> s2 = np_sum<Sum2<double>, SM>(f2, m);
    corr = s2.a / (double)m;
    mse = s2.b / (double)m;
  } else {
    auto fp = [&](int k) -> double { return side_z(q, k) * side_z(c, k); };
    corr = np_sum<double, SM>(fp, m) / (double)m;                                  // :154
    auto fd = [&](int k) -> double { double d = q.x[k] - c.x[k]; return d * d; };
    mse = np_sum<double, SM>(fd, m) / (double)m;                                   // :161
  }
  const double sim = (corr + 1.0) / 2.0;                                         // :158
  const double maxmse = q.msq + c.msq;                                           // :162
  double ds = 1.0;
  if (maxmse > 0.0) {
    ds = 1.0 - (mse / maxmse);
    ds = ds > 0.0 ? ds : 0.0;
  }
  const double a = 0.7 * sim;
  const double b = 0.3 * ds;
  double comb = a + b;                                                           // :171
  comb = comb < 1.0 ? comb : 1.0;
  return comb > 0.0 ? comb : 0.0;
}

template <bool SM = false, bool F2 = false>
__device__ double exact_level(const double* q, const double* zq, const double* sq, const double* c,
                              const double* zc, const double* sc, int m, int* np32) {
  const bool qf = (aux_bits(sq) & kAuxF32) != 0, cf = (aux_bits(sc) & kAuxF32) != 0;
  return exact_level_sides<SM, F2>(make_side<SM>(q, zq, sq, m, qf), make_side<SM>(c, zc, sc, m, cf), m, np32);
}

// exact_pair on explicit row pointers (raw [L], Z [Lp], S [nseg x 4] of each side; global or LDS)
// typed (level >= 0, nullable): 1 when the level score is a numpy float32 (the reference's threshold test
// then compares in float32, NEP 50: see typed_pass)
template <bool SM = false, bool F2 = false>
__device__ double exact_pair_rows(const double* ra, const double* za, const double* sa, const double* rb,
                                  const double* zb, const double* sb, const SegInfo& si, int level, double* lv,
                                  int* typed = nullptr) {
  int t32;
  if (level >= 0) {
    if (level >= si.nseg) return 0.0;
    const int s = level;
    const double v = exact_level<SM, F2>(ra + si.src[s], za ? za + si.poff[s] : nullptr, sa + 4 * s, rb + si.src[s],
                                     zb ? zb + si.poff[s] : nullptr, sb + 4 * s, si.len[s], &t32);
    if (typed) *typed = t32;
    return v;
  }
  // search_engine.py:191-230: running weighted sum in level order, divide, clamp.  Python typing:
  // the sum starts as the Python float 0.0; a float32 level score makes the term float32 (the weight
  // is cast to float32) and from then on the sum is float32 (a Python float operand is cast to it).
  double tws = 0.0, tw = 0.0;
  bool acc32 = false;
  for (int s = 0; s < si.nseg; ++s) {
    const double v = exact_level<SM, F2>(ra + si.src[s], za ? za + si.poff[s] : nullptr, sa + 4 * s, rb + si.src[s],
                                     zb ? zb + si.poff[s] : nullptr, sb + 4 * s, si.len[s], &t32);
    if (lv) lv[s] = v;
    const double w = 1.0 / (double)(s + 1);
    const double term = t32 ? (double)((float)v * (float)w) : v * w;
    if (!acc32 && !t32) {
      tws = tws + term;
    } else {
      tws = (double)((float)tws + (float)term);
      acc32 = true;
    }
    tw = tw + w;
  }
  double ov;
  if (acc32) {
    const float o = (float)tws / (float)tw;
    ov = o < 1.0f ? (double)o : 1.0;
  } else {
    ov = tw > 0.0 ? tws / tw : 0.0;
    ov = ov < 1.0 ? ov : 1.0;
  }
  return ov > 0.0 ? ov : 0.0;
}

// ZB = false: B's normalised values are recomputed from its raw values and statistics ((x - mean) / std
// in f64, the exact operation that wrote Z: bit-identical), so B's Z rows are not read — the re-rank and
// re-score kernels read only the candidates' raw rows and statistics (half the bytes of a row pair)
template <bool SM = false, bool ZB = true, bool F2 = false>
__device__ double exact_pair(const VecSet& A, int64_t ia, const VecSet& B, int64_t ib, const SegInfo& si, int level,
                             double* lv, int* typed = nullptr) {
  return exact_pair_rows<SM, F2>(A.raw + ia * si.L, A.Z + ia * si.Lp, A.S + ia * si.nseg * 4, B.raw + ib * si.L,
                             ZB ? B.Z + ib * si.Lp : nullptr, B.S + ib * si.nseg * 4, si, level, lv, typed);
}

// The reference's threshold test of a level score (search_engine.py:284-292 `>=`, video_search.py:244 `>`)
// with Python typing: a numpy float32 score is compared with the Python-float threshold in float32
// (NEP 50: the threshold is rounded to float32), a Python-float score in float64.  Callers pass the
// threshold as given (f32_threshold, hq_mi355x core/search_engine.py, folds the rounding into one value
// only for all-float32 pools; this per-pair form also covers pools mixing float32 and float64 vectors).
__device__ __forceinline__ bool typed_pass(double e, int typed, double thr, int thr_mode) {
  if (thr_mode == 0) return true;
  const double t = typed ? (double)(float)thr : thr;
  return thr_mode == 1 ? e >= t : e > t;
}
// lowest threshold any pair is tested against (the completeness proofs must hold for both typings)
__device__ __forceinline__ double thr_low(double thr) {
  const double t32 = (double)(float)thr;
  return t32 < thr ? t32 : thr;
}

// Sort keys of all-float32 searches (thr_mode | kThrKey32 on the re-rank, flag 1 of hq_progressive_final_ex):
// the reference sorts a list mixing numpy float32 scores and Python-float scores (constant branches, clamps;
// core/search_engine.py:291, :387), and NumPy 2 (NEP 50) compares the two in float32, so float32(0.1) ties a
// Python 0.1 and the stable sort keeps their pool order.  The Python floats there are the constant-branch
// values and their weighted means, which float32 rounding keeps distinct, so ranking by the float32-rounded
// value reproduces Python's order exactly.  A list is then proven complete when float32(last approximate
// + eps) < float32(k-th exact): an unlisted pair's key is at most the former.
constexpr int kThrKey32 = 8;
__device__ __forceinline__ double key_of(double x, bool k32) { return k32 ? (double)(float)x : x; }

// dense Q x N exact scores (drop-in path and rare exact fallbacks)
template <bool SM = false>
__global__ __launch_bounds__(256) void k_level_scores(VecSet Qs, int Q, VecSet Cs, int64_t N, SegInfo si, int level,
                                                      double* __restrict__ out) {
  const int64_t total = (int64_t)Q * N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / N, c = t % N;
    out[t] = exact_pair<SM>(Qs, q, Cs, c, si, level, nullptr);
  }
}

// Dense exact level scores with coalesced candidate rows (level >= 0, segments of <= 128 values): a block
// of kLsTile threads stages the level segment of kLsTile consecutive candidate rows into LDS (consecutive
// threads read consecutive values of a row: 256-B runs instead of one row per thread), then thread t
// scores candidate c0 + t against the block's kLsQ queries from LDS.  The same exact_level code on other
// addresses (the candidate's normalised values recomputed as (x - mean) / std, the f64 operations
// k_seg_prepare stored in Z), so the scores are bit-identical to k_level_scores.
constexpr int kLsTile = 128, kLsQ = 4;
__global__ __launch_bounds__(kLsTile) void k_level_scores_lds(VecSet Qs, int Q, VecSet Cs, int64_t N, SegInfo si,
                                                              int level, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double lsm[];
  const int m = si.len[level], src = si.src[level], pitch = m | 1;  // odd pitch: conflict-free row reads
  const int64_t c0 = (int64_t)blockIdx.x * kLsTile;
  const int q0 = blockIdx.y * kLsQ;
  const int tid = threadIdx.x;
  const int nrow = N - c0 < kLsTile ? (int)(N - c0) : kLsTile;
  for (int e = tid; e < nrow * m; e += kLsTile) {
    const int r = e / m, k = e - r * m;
    lsm[r * pitch + k] = Cs.raw[(c0 + r) * si.L + src + k];
  }
  __syncthreads();
  if (tid >= nrow) return;
  const int64_t c = c0 + tid;
  const double* rc = lsm + tid * pitch;
  const double* sc = Cs.S + (c * si.nseg + level) * 4;
  for (int qi = 0; qi < kLsQ && q0 + qi < Q; ++qi) {
    const int64_t q = q0 + qi;
    int t32;
    out[q * N + c] = exact_level<true>(Qs.raw + q * si.L + src, Qs.Z + q * si.Lp + si.poff[level],
                                       Qs.S + (q * si.nseg + level) * 4, rc, nullptr, sc, m, &t32);
  }
}

// exact overall + per-level for selected (query, candidate) pairs; ids are global, id_base subtracted.
// G lanes per pair (G >= nseg): lane s computes level s, the pair's first lane adds them up in level
// order with the reference's typing (exact_pair's sum), so the 5-7 level scores run in parallel.
template <int G, bool SM = false, bool ZC = true>
__global__ __launch_bounds__(256) void k_rescore(VecSet Qs, int Q, VecSet Cs, int64_t N, SegInfo si,
                                                 const int64_t* __restrict__ ids, int k, int64_t id_base,
                                                 double* __restrict__ out) {
  const int64_t total = (int64_t)Q * k;
  const int W = 1 + si.nseg;
  const int sub = threadIdx.x % G;
  for (int64_t t0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G; t0 < total;
       t0 += ((int64_t)gridDim.x * blockDim.x) / G) {
    const int64_t t = t0;
    const int64_t q = t / k;
    const int64_t gid = ids[t];
    double* o = out + t * W;
    const int64_t c = gid - id_base;
    const bool ok = !(gid < 0 || c < 0 || c >= N);
    double v = 0.0;
    int t32 = 0;
    if (ok && sub < si.nseg) {
      const int s = sub;
      v = exact_level<SM>(Qs.raw + q * si.L + si.src[s], Qs.Z + q * si.Lp + si.poff[s], Qs.S + (q * si.nseg + s) * 4,
                      Cs.raw + c * si.L + si.src[s], ZC ? Cs.Z + c * si.Lp + si.poff[s] : nullptr,
                      Cs.S + (c * si.nseg + s) * 4, si.len[s], &t32);
    }
    if (sub < si.nseg) o[1 + sub] = v;
    // search_engine.py:191-230 typed running sum (see exact_pair), gathered from the group's lanes
    double tws = 0.0, tw = 0.0;
    bool acc32 = false;
    for (int s = 0; s < si.nseg; ++s) {
      const int src = (threadIdx.x & 63) - sub + s;
      const double vs = __shfl(v, src, 64);
      const int ts = __shfl(t32, src, 64);
      const double w = 1.0 / (double)(s + 1);
      const double term = ts ? (double)((float)vs * (float)w) : vs * w;
      if (!acc32 && !ts) {
        tws = tws + term;
      } else {
        tws = (double)((float)tws + (float)term);
        acc32 = true;
      }
      tw = tw + w;
    }
    if (sub == 0) {
      double ov;
      if (!ok) {
        ov = 0.0;
      } else if (acc32) {
        const float of = (float)tws / (float)tw;
        ov = of < 1.0f ? (double)of : 1.0;
        ov = ov > 0.0 ? ov : 0.0;
      } else {
        ov = tw > 0.0 ? tws / tw : 0.0;
        ov = ov < 1.0 ? ov : 1.0;
        ov = ov > 0.0 ? ov : 0.0;
      }
      o[0] = ov;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// fused scan: MFMA f64 contraction + epilogue + per-query top-k (score desc, id asc)
// WG = 4 waves; 64 queries (16 per wave) x one corpus chunk, 64 candidates per step.
// ------------------------------------------------------------------------------------------------
constexpr int kQB = 64;       // queries per workgroup
constexpr int kCB = 64;       // candidates per step
constexpr int kMaxTopK = 64;
constexpr int kMaxFinal = 256;  // survivors handled by k_progressive_final

struct ScanArgs {
  const double* Zq; const double* Sq; int Q;
  const double* Zc; const double* Sc; int64_t N;
  SegInfo si;
  int ks;          // k-steps (4 f64 each) processed: level0 -> plen[0]/4, overall -> Lp/4
  int nseg_used;   // 1 (level0) or nseg (overall)
  int rs;          // LDS row stride of the candidate tile (f64), == 2 mod 32, >= 4*ks
  int K;           // top-k
  double thr; int thr_mode;  // 0 none, 1 >=, 2 >
  int64_t id_base;
  int64_t chunk_len; int nchunks; int nqb;
  double* ws_score; int64_t* ws_id; double* ws_best; int64_t* ws_best_id;
};

__device__ __forceinline__ bool better(double s, int64_t id, double s2, int64_t id2) {
  return s > s2 || (s == s2 && id < id2);
}

template <int KSMAX, bool OVERALL>
__global__ __launch_bounds__(256) void k_scan(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nsu = a.nseg_used;
  // LDS carve
  double* btile = reinterpret_cast<double*>(smem);                         // kCB x rs
  double* cstat = btile + kCB * a.rs;                                      // kCB x nsu x 4
  double* qstat = cstat + kCB * nsu * 4;                                   // kQB x nsu x 4
  double* stile = qstat + kQB * nsu * 4;                                   // 4 x 16 x kCB
  double* lscore = stile + 4 * 16 * kCB;                                   // kQB x K
  int64_t* lid = reinterpret_cast<int64_t*>(lscore + kQB * a.K);           // kQB x K
  unsigned long long* mask = reinterpret_cast<unsigned long long*>(lid + kQB * a.K);  // kQB
  double* tau = reinterpret_cast<double*>(mask + kQB);                     // kQB
  int* lcnt = reinterpret_cast<int*>(tau + kQB);                           // kQB

  // XCD-aware block -> (query block, chunk): the nqb blocks of one chunk share an XCD (same
  // blockIdx % 8) and are dispatched back to back, so the chunk's candidate tiles come from L2.
  const int b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.N) c_end = a.N;

  const int qw0 = qb * kQB + wave * 16;  // first query of this wave
  const SegInfo& si = a.si;

  // A fragments (kept in registers for the whole chunk): lane holds Zq[qw0 + (lane&15)][4t + (lane>>4)]
  double af[KSMAX];
  {
    const int q = qw0 + (lane & 15);
#pragma unroll
    for (int t = 0; t < KSMAX; ++t) {
      double v = 0.0;
      if (t < a.ks && q < a.Q) v = a.Zq[(int64_t)q * si.Lp + 4 * t + (lane >> 4)];
      af[t] = v;
    }
  }
  // query stats -> LDS, list init
  for (int i = tid; i < kQB * nsu; i += 256) {
    const int ql = i / nsu, s = i % nsu;
    const int q = qb * kQB + ql;
    for (int j = 0; j < 4; ++j) qstat[i * 4 + j] = (q < a.Q) ? a.Sq[((int64_t)q * si.nseg + s) * 4 + j] : 1.0;
  }
  for (int i = tid; i < kQB; i += 256) {
    mask[i] = 0ull;
    tau[i] = -__builtin_huge_val();
    lcnt[i] = 0;
  }
  for (int i = tid; i < kQB * a.K; i += 256) {
    lscore[i] = -__builtin_huge_val();
    lid[i] = -1;
  }
  // lane's best (first arg-max) for its 4 query rows
  double best[4];
  int64_t best_id[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { best[r] = -__builtin_huge_val(); best_id[r] = -1; }
  __syncthreads();

  const int pieces_per_row = 2 * a.ks;  // 16-byte pieces of the used K columns
  const int npieces = kCB * pieces_per_row;
  const int nstat = kCB * nsu * 4;
  // register prefetch of the next candidate tile (software pipelining) for the short-K scans
  constexpr bool PREF = KSMAX <= 16;
  constexpr int PMAX = PREF ? (kCB * 2 * KSMAX + 255) / 256 : 1;
  constexpr int SMAX = PREF ? (kCB * 4 + 255) / 256 : 1;
  double2 pf[PMAX];
  double ps[SMAX];
  auto fetch = [&](int64_t cs) {
#pragma unroll
    for (int u = 0; u < PMAX; ++u) {
      const int p = tid + 256 * u;
      double2 v = make_double2(0.0, 0.0);
      if (p < npieces) {
        const int c = p / pieces_per_row, kk = p % pieces_per_row;
        const int64_t gc = cs + c;
        if (gc < c_end) v = *reinterpret_cast<const double2*>(a.Zc + gc * si.Lp + 2 * kk);
      }
      pf[u] = v;
    }
#pragma unroll
    for (int u = 0; u < SMAX; ++u) {
      const int i = tid + 256 * u;
      double v = 1.0;
      if (i < nstat) {
        const int c = i / 4, j = i % 4;  // nsu == 1 on this path
        const int64_t gc = cs + c;
        if (gc < c_end) v = a.Sc[gc * si.nseg * 4 + j];
      }
      ps[u] = v;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < PMAX; ++u) {
      const int p = tid + 256 * u;
      if (p < npieces) {
        const int c = p / pieces_per_row, kk = p % pieces_per_row;
        *reinterpret_cast<double2*>(btile + c * a.rs + 2 * kk) = pf[u];
      }
    }
#pragma unroll
    for (int u = 0; u < SMAX; ++u) {
      const int i = tid + 256 * u;
      if (i < nstat) cstat[i] = ps[u];
    }
  };
  if (PREF && nsu == 1 && c_begin < c_end) fetch(c_begin);
  for (int64_t cs = c_begin; cs < c_end; cs += kCB) {
    // ---- stage candidate tile + stats -------------------------------------------------------
    if (PREF && nsu == 1) {
      stash();
    } else {
      for (int p = tid; p < npieces; p += 256) {
        const int c = p / pieces_per_row, kk = p % pieces_per_row;
        const int64_t gc = cs + c;
        double2 v = make_double2(0.0, 0.0);
        if (gc < c_end) v = *reinterpret_cast<const double2*>(a.Zc + gc * si.Lp + 2 * kk);
        *reinterpret_cast<double2*>(btile + c * a.rs + 2 * kk) = v;
      }
      for (int i = tid; i < kCB * nsu; i += 256) {
        const int c = i / nsu, s = i % nsu;
        const int64_t gc = cs + c;
        for (int j = 0; j < 4; ++j) cstat[i * 4 + j] = (gc < c_end) ? a.Sc[(gc * si.nseg + s) * 4 + j] : 1.0;
      }
    }
    __syncthreads();
    if (PREF && nsu == 1 && cs + kCB < c_end) fetch(cs + kCB);  // next tile in flight during compute

    // ---- contraction + epilogue ---------------------------------------------------------------
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int cl = cb * 16 + (lane & 15);        // candidate column of this lane
      const double* brow = btile + cl * a.rs + (lane >> 4);
      double score[4];
      if constexpr (!OVERALL) {
        dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int t = 0; t < KSMAX; ++t)
          if (t < a.ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t], brow[4 * t], acc, 0, 0, 0);
        const double* cst = cstat + cl * nsu * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double* qst = qstat + (wave * 16 + (lane >> 4) + 4 * r) * nsu * 4;
          score[r] = level_sim(acc[r], qst[0], qst[1], qst[2], cst[0], cst[1], cst[2], (double)si.len[0],
                               si.inv_m[0], (aux_bits(qst) & aux_bits(cst) & kAuxF32) != 0);
        }
      } else {
        double tws[4] = {0.0, 0.0, 0.0, 0.0};
        for (int s = 0; s < si.nseg; ++s) {
          dbl4 acc = {0.0, 0.0, 0.0, 0.0};
          const int t0 = si.poff[s] >> 2, t1 = (si.poff[s] + si.plen[s]) >> 2;
#pragma unroll
          for (int t = 0; t < KSMAX; ++t)
            if (t >= t0 && t < t1) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t], brow[4 * t], acc, 0, 0, 0);
          const double* cst = cstat + (cl * nsu + s) * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double* qst = qstat + ((wave * 16 + (lane >> 4) + 4 * r) * nsu + s) * 4;
            double v = level_sim(acc[r], qst[0], qst[1], qst[2], cst[0], cst[1], cst[2], (double)si.len[s],
                                 si.inv_m[s], (aux_bits(qst) & aux_bits(cst) & kAuxF32) != 0);
            tws[r] = tws[r] + v * si.w[s];
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double ov = tws[r] / si.wsum;
          ov = ov < 1.0 ? ov : 1.0;
          score[r] = ov > 0.0 ? ov : 0.0;
        }
      }
      const int64_t cid = cs + cl;
      const bool cvalid = cid < c_end;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = wave * 16 + (lane >> 4) + 4 * r;  // query row inside the WG
        const bool qvalid = qb * kQB + ql < a.Q;
        const double s = score[r];
        if (cvalid && qvalid) {
          if (s > best[r]) { best[r] = s; best_id[r] = cid; }
          const bool thr_ok = a.thr_mode == 0 || (a.thr_mode == 1 ? s >= a.thr : s > a.thr);
          if (thr_ok && s > tau[ql]) {
            stile[(wave * 16 + ((lane >> 4) + 4 * r)) * kCB + cl] = s;
            atomicOr(&mask[ql], 1ull << cl);
          }
        }
      }
    }
    __syncthreads();

    // ---- merge passing candidates into the sorted per-query lists, one wave per query ---------
    // (lists sorted by (score desc, id asc); a candidate's slot = #entries better than it, found with
    // one ballot; the tail shifts by one lane)
    for (int qq = 0; qq < 16; ++qq) {
      const int ql = wave * 16 + qq;
      unsigned long long m = mask[ql];
      if (m == 0ull) continue;
      double es = lane < a.K ? lscore[ql * a.K + lane] : -__builtin_huge_val();
      int64_t ei = lane < a.K ? lid[ql * a.K + lane] : -1;
      while (m) {
        const int bit = __builtin_ctzll(m);
        m &= m - 1;
        const double sc = stile[ql * kCB + bit];
        const int64_t id = cs + bit;
        const bool bt = (ei >= 0) && better(es, ei, sc, id);
        const int p = __popcll(__ballot(bt));
        if (p >= a.K) continue;
        const double us = __shfl_up(es, 1, 64);
        const int64_t ui = __shfl_up(ei, 1, 64);
        if (lane > p) { es = us; ei = ui; }
        if (lane == p) { es = sc; ei = id; }
      }
      if (lane < a.K) {
        lscore[ql * a.K + lane] = es;
        lid[ql * a.K + lane] = ei;
      }
      const double wsc = __shfl(es, a.K - 1, 64);
      const int64_t wid = __shfl(ei, a.K - 1, 64);
      if (lane == 0) {
        tau[ql] = wid >= 0 ? wsc : -__builtin_huge_val();
        mask[ql] = 0ull;
      }
    }
    __syncthreads();
  }

  // ---- write this chunk's lists and arg-max ---------------------------------------------------
  for (int i = tid; i < kQB * a.K; i += 256) {
    const int ql = i / a.K, j = i % a.K;
    const int q = qb * kQB + ql;
    if (q >= a.Q) continue;
    const int64_t o = ((int64_t)chunk * a.Q + q) * a.K + j;
    if (lid[ql * a.K + j] >= 0) {
      a.ws_score[o] = lscore[ql * a.K + j];
      a.ws_id[o] = lid[ql * a.K + j] + a.id_base;
    } else {
      a.ws_score[o] = -__builtin_huge_val();
      a.ws_id[o] = -1;
    }
  }
  // reduce best across the 16 lanes sharing (lane >> 4): xor over the low 4 lane bits
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double s = best[r];
    int64_t id = best_id[r];
    for (int o = 1; o < 16; o <<= 1) {
      const double s2 = __shfl_xor(s, o, 64);
      const int64_t id2 = __shfl_xor(id, o, 64);
      if (id2 >= 0 && (id < 0 || better(s2, id2, s, id))) { s = s2; id = id2; }
    }
    const int q = qw0 + (lane >> 4) + 4 * r;
    if ((lane & 15) == 0 && q < a.Q) {
      a.ws_best[(int64_t)chunk * a.Q + q] = s;
      a.ws_best_id[(int64_t)chunk * a.Q + q] = id >= 0 ? id + a.id_base : -1;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// level-0 scan, wave-independent (the progressive search's filtering stage; k_scan handles the
// overall mode and the arg-max).  One wave = 64 queries (4 MFMA column blocks of 16) x one corpus
// chunk, 16 candidates per step:
//   D[cand][query] = sum_k Zc[cand][k] Zq[query][k] with v_mfma_f64_16x16x4f64, A = candidates,
//   B = queries.  Lane group g = lane >> 4 feeds the contiguous k range [g*KS, g*KS + KS), so each
//   lane loads its candidate fragment with KS/2 16-byte loads straight from HBM/L2 (no LDS staging,
//   no barriers); the query fragments stay in registers for the whole chunk.
// Lane (g, j) owns queries 16b + j (b < 4) and candidates g + 4r (r < 4) of the step.
// Filter without division: with base = 0.35 + 0.35 G/m, num = 0.6 (qs cs G / m + qm cm) and
// den = msq_q + msq_c, score >= th  <=>  th - base <= 0  or  num >= (th - base) den.
// th(query) = max(threshold, own K-th best, best K-th of any other wave for that query); the last
// is exchanged through a per-query atomicMax in global memory (scores >= 0 order like their bit
// patterns), so after the first chunks almost nothing reaches the insert path.  Every pruned
// candidate is below the K-th best of some complete list, so the merged top-K is unchanged.
// ------------------------------------------------------------------------------------------------
constexpr int kQW = 64;  // queries per wave
constexpr int kCS = 16;  // candidates per step

struct Scan0Args {
  const double* Zq; const double* Sq; int Q;
  const double* Zc; const double* Sc; int64_t N;
  const float* Zq32; const float* Zc32;  // f64 kernels: unused
  const _Float16* Zq16; const _Float16* Zc16;  // split kernels: level-0 rows [hi 32 | lo 32] (+kPad0 rows)
  const float* Sq32; const float* Sc32;  // split kernels: level-0 (std, mean, msq, flag bits) per row
  int Lp, nseg, P0;
  double inv_m, c1;  // 1/m, 0.35/m
  int K;
  double thr0;       // initial threshold (-inf: none)
  const double* th0; // per-query lower bound of the K-th best approximate score (sample pass) or null
  int64_t id_base;
  int64_t chunk_len; int nchunks; int nqb;
  double* ws_score; int64_t* ws_id; unsigned long long* gtau;
  float* pool_s; int* pool_i; int* pool_n; int pool_cap;  // k_scan0f: per-query candidate pools
  const void* qconst; // k_scan0g: per-query QConst table (k_sample_kth / k_scan_qprep)
  int expt;          // HQ_SCAN_EXPT=3: count insert-path entries, passing pairs and list merges
  unsigned long long* dbg;  // expt 3: [entries, passing pairs, list inserts]
};

__device__ __forceinline__ double rl_f64(double v, int l) {
  const int2 p = *reinterpret_cast<int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_readlane(p.x, l);
  r.y = __builtin_amdgcn_readlane(p.y, l);
  return *reinterpret_cast<double*>(&r);
}

// lane i <- lane i-1 (lane 0 keeps its own value): DPP wave_shr:1
__device__ __forceinline__ int shr1_i32(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ double shr1_f64(double v) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = shr1_i32(p.x);
  p.y = shr1_i32(p.y);
  return *reinterpret_cast<double*>(&p);
}

// approximate level-0 score of a pair with both stds non-zero (the insert path and the sample pass
// use this same expression, so their values agree bit for bit)
__device__ __forceinline__ double approx0(double G, double c1, double qA, double qB, double qQ, double cs, double cm,
                                          double cq) {
  const double base = fma(G, c1, 0.35);
  const double num = fma(G, qA * cs, qB * cm);
  double t = num / (qQ + cq);
  t = t > 0.0 ? t : 0.0;
  double s = base + t;
  s = s < 1.0 ? s : 1.0;
  return s > 0.0 ? s : 0.0;
}

typedef float flt4 __attribute__((ext_vector_type(4)));
typedef float flt2 __attribute__((ext_vector_type(2)));

// Z operand type of the f64 contraction (v_mfma_f64_16x16x4f64, C/D row (lane>>4) + 4r).
template <bool F32> struct ZOps;
template <> struct ZOps<false> {
  typedef double T;
  typedef dbl4 Acc;
  static __device__ __forceinline__ Acc mfma(T a, T b, Acc c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  static __device__ __forceinline__ int row(int g, int r) { return g + 4 * r; }
  static __device__ __forceinline__ const T* zq(const Scan0Args& a, int64_t q) { return a.Zq + q * a.Lp; }
  static __device__ __forceinline__ const T* zc(const Scan0Args& a, int64_t c) { return a.Zc + c * a.Lp; }
};

#ifdef HQ_DIAG
// f64 sources only (hq_seg_prepare without float32 rows): the constant branch compares means in f64
template <int KS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_scan0(Scan0Args a) {
  typedef ZOps<false> Z;
  typedef typename Z::T ZT;
  typedef typename Z::Acc AccT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  double* qc = reinterpret_cast<double*>(smem);      // kQW x 4: 0.6 qs / m, 0.6 qm, msq, mean
  double* ls = qc + kQW * 4;                          // kQW x K approx scores
  int* li = reinterpret_cast<int*>(ls + kQW * a.K);   // kQW x K corpus rows
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.N) c_end = a.N;
  const int q0 = qb * kQW;
  const int K = a.K;

  // query fragments (registers, whole chunk), constants (LDS), thresholds (registers)
  ZT qf[4][KS];
  double th[4];
  int qz = 0;  // bit b: query 16b + j has zero std
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const ZT* zr = Z::zq(a, v ? q : 0) + g * KS;
#pragma unroll
    for (int t = 0; t < KS; ++t) qf[b][t] = v ? zr[t] : (ZT)0;
    const double* st = a.Sq + (int64_t)(v ? q : 0) * a.nseg * 4;
    const double qm = st[0], qs = st[1], qq = st[2];
    if (g == 0) {
      double* c = qc + (16 * b + j) * 4;
      c[0] = (0.6 * a.inv_m) * qs;
      c[1] = 0.6 * qm;
      c[2] = qq;
      c[3] = qm;
    }
    double t0 = a.thr0;
    if (v && a.th0 && a.th0[q] > t0) t0 = a.th0[q];
    th[b] = v ? t0 : __builtin_huge_val();
    if (v && qs == 0.0) qz |= 1 << b;
  }
  for (int i = lane; i < kQW * K; i += 64) {
    ls[i] = -__builtin_huge_val();
    li[i] = -1;
  }
  const bool myq = q0 + lane < a.Q;  // lane's query for the global-threshold exchange

  // candidate fragment of a step: row cs + j, k range [g*KS, g*KS + KS)
  typedef double dbl2v __attribute__((ext_vector_type(2)));
  auto load_frag = [&](int64_t cs, ZT* dst) {
    int64_t c = cs + j;
    if (c >= c_end) c = c_end - 1;
    const ZT* p = Z::zc(a, c) + g * KS;
    constexpr int W = 16 / sizeof(ZT);  // elements per 16-byte load
    if constexpr ((KS % W) == 0) {
      typedef ZT vec __attribute__((ext_vector_type(16 / sizeof(ZT))));
#pragma unroll
      for (int t = 0; t < KS; t += W) {
        const vec v = *reinterpret_cast<const vec*>(p + t);
#pragma unroll
        for (int e = 0; e < W; ++e) dst[t + e] = v[e];
      }
    } else {
#pragma unroll
      for (int t = 0; t < KS; ++t) dst[t] = p[t];
    }
  };
  // candidate statistics of a step for the lane's rows Z::row(g, r): mean, std, msq
  auto load_stats = [&](int64_t cs, double* dst) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int64_t c = cs + Z::row(g, r);
      if (c >= c_end) c = c_end - 1;
      const double* st = a.Sc + c * a.nseg * 4;
      const dbl2v v = *reinterpret_cast<const dbl2v*>(st);
      dst[3 * r] = v.x;
      dst[3 * r + 1] = v.y;
      dst[3 * r + 2] = st[2];
    }
  };
  // MFMAs of one half (two 16-query blocks) of a step
  auto mfma_half = [&](const int h, const ZT* f, AccT* acc) {
    acc[0] = AccT{0, 0, 0, 0};
    acc[1] = AccT{0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < KS; ++t) {  // two interleaved chains
      acc[0] = Z::mfma(f[t], qf[2 * h][t], acc[0]);
      acc[1] = Z::mfma(f[t], qf[2 * h + 1][t], acc[1]);
    }
  };
  // filter of one half of the step starting at row cs: branch-free, so the scheduler can interleave
  // it with the other half's MFMAs.  Returns the lane's pass bits (bit 4u + r).
  auto filter_half = [&](const int h, const AccT* acc, const int64_t cs, const double* cst,
                         double* qa, double* qbv, double* qqv) -> int {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const double* c = qc + (16 * (2 * h + u) + j) * 4;
      const dbl2v v0 = *reinterpret_cast<const dbl2v*>(c);
      qa[u] = v0.x;
      qbv[u] = v0.y;
      qqv[u] = c[2];
    }
    int bits = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool inval = cs + Z::row(g, r) >= c_end;
      const bool zc = cst[3 * r + 1] == 0.0;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int b = 2 * h + u;
        const double G = (double)acc[u][r];
        const double R = th[b] - fma(G, a.c1, 0.35);
        const double num = fma(G, qa[u] * cst[3 * r + 1], qbv[u] * cst[3 * r]);
        const double den = qqv[u] + cst[3 * r + 2];
        // zero-variance pairs go to the insert path, which evaluates and tests them exactly;
        // rows past the chunk end never pass
        const bool spec = zc | (((qz >> b) & 1) != 0);
        const bool p = ((R <= 0.0) | (num >= R * den) | spec) & !inval;
        bits |= (int)p << (4 * u + r);
      }
    }
    return bits;
  };
  // insert the passing pairs of one half (rare once the thresholds are up)
  auto insert_half = [&](const int h, const AccT* acc, const int64_t cs, const double* cst, const double* qa,
                         const double* qbv, const double* qqv, const int bits) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 2 * h + u;
        unsigned long long m = __ballot((bits >> (4 * u + r)) & 1);
        if (m == 0ull) continue;
        const double csd = cst[3 * r + 1], cm = cst[3 * r];
        const bool zq = (qz >> b) & 1, zc = csd == 0.0;
        const double s = (zq || zc) ? const0(zq, zc, qc[(16 * b + j) * 4 + 3], cm)
                                    : approx0((double)acc[u][r], a.c1, qa[u], qbv[u], qqv[u], csd, cm, cst[3 * r + 2]);
        while (m) {
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          const int c_off = Z::row(l >> 4, r);
          const double sc = rl_f64(s, l);
          if (!(sc >= rl_f64(th[b], l))) continue;
          const int qi = 16 * b + (l & 15);
          const int id = (int)(cs + c_off);
          double es = lane < K ? ls[qi * K + lane] : -__builtin_huge_val();
          int ei = lane < K ? li[qi * K + lane] : -1;
          const bool bt = (ei >= 0) && (es > sc || (es == sc && ei < id));
          const int p = __popcll(__ballot(bt));
          if (p >= K) continue;
          const double us = shr1_f64(es);
          const int ui = shr1_i32(ei);
          if (lane > p) { es = us; ei = ui; }
          if (lane == p) { es = sc; ei = id; }
          if (lane < K) {
            ls[qi * K + lane] = es;
            li[qi * K + lane] = ei;
          }
          if (__builtin_amdgcn_readlane(ei, K - 1) >= 0) {
            const double tau = rl_f64(es, K - 1);
            if (j == (l & 15)) th[b] = tau > th[b] ? tau : th[b];
            if (lane == 0 && tau > 0.0)
              atomicMax(a.gtau + q0 + qi, (unsigned long long)__double_as_longlong(tau));
          }
        }
      }
  };
  // 16 MFMAs interleaved with the filter's VALU work
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
    }
  };

  // Software pipeline: the MFMAs of one half run while the VALU filters the other half
  //   block A: MFMA(step i, half 1)   || filter(step i, half 0)
  //   block B: MFMA(step i+1, half 0) || filter(step i, half 1)
  ZT cf[KS];
  double cst[12];
  load_frag(c_begin, cf);
  load_stats(c_begin, cst);
  AccT acc0[2], acc1[2];
  mfma_half(0, cf, acc0);
  unsigned long long gt_bits = 0ull;
  int step = 0;
  for (int64_t cs = c_begin; cs < c_end; cs += kCS, ++step) {
    ZT cfn[KS];
    double cstn[12];
    load_frag(cs + kCS, cfn);  // unconditional (rows clamp to the chunk): keeps the wait counts exact
    load_stats(cs + kCS, cstn);
    double qa[2], qbv[2], qqv[2];
    mfma_half(1, cf, acc1);
    const int bits0 = filter_half(0, acc0, cs, cst, qa, qbv, qqv);
    interleave();
    if (__ballot(bits0 != 0)) insert_half(0, acc0, cs, cst, qa, qbv, qqv, bits0);
    mfma_half(0, cfn, acc0);  // next step's first half (a harmless repeat of the last row at the end)
    const int bits1 = filter_half(1, acc1, cs, cst, qa, qbv, qqv);
    interleave();
    if (__ballot(bits1 != 0)) insert_half(1, acc1, cs, cst, qa, qbv, qqv, bits1);
#pragma unroll
    for (int t = 0; t < KS; ++t) cf[t] = cfn[t];
#pragma unroll
    for (int t = 0; t < 12; ++t) cst[t] = cstn[t];
    // ---- global thresholds, every 4 steps (applied from the next step) ----
    if ((step & 3) == 0) {
      if (gt_bits != 0ull) {
        const double gd = __longlong_as_double((long long)gt_bits);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const double v = __shfl(gd, 16 * b + j, 64);
          th[b] = v > th[b] ? v : th[b];
        }
      }
      if (myq) gt_bits = __atomic_load_n(a.gtau + q0 + lane, __ATOMIC_RELAXED);
    }
  }

  // ---- this chunk's lists ----
  for (int i = lane; i < kQW * K; i += 64) {
    const int ql = i / K, jj = i % K;
    const int q = q0 + ql;
    if (q >= a.Q) continue;
    const int64_t o = ((int64_t)chunk * a.Q + q) * K + jj;
    const int id = li[i];
    a.ws_score[o] = id >= 0 ? ls[i] : -__builtin_huge_val();
    a.ws_id[o] = id >= 0 ? (int64_t)id + a.id_base : -1;
  }
}
#endif  // HQ_DIAG

// ------------------------------------------------------------------------------------------------
// sample pass for k_scan0: a strided subset of the corpus (row i*stride) is scored with the same
// MFMA contraction and the same approximate-score expression; each query gets a 256-bin histogram of
// its sample scores over [0, 1].  The highest bin edge e/256 with >= K sample scores at or above it
// is a lower bound of the K-th best score over the whole corpus (the sample is a subset), which
// k_scan0 uses as its starting threshold, so only ~stride*K candidates per query reach its lists.
// ------------------------------------------------------------------------------------------------
constexpr int kBins = 256;

struct SampleArgs {
  const double* Zq; const double* Sq; int Q;
  const double* Zc; const double* Sc; int64_t N;
  const float* Zq32; const float* Zc32;
  const _Float16* Zq16; const _Float16* Zc16;
  const float* Sq32; const float* Sc32;
  int Lp, nseg, P0;
  double inv_m, c1;
  int64_t stride, S;
  int64_t chunk_len; int nchunks; int nqb;
  int K;
  unsigned int* hist;  // Q x kBins
  float* top;          // k_sample_topf: Q x 4 nchunks x kTopT
};

#ifdef HQ_DIAG
constexpr int kHRow = kBins / 2 + 1;  // LDS words per query histogram (odd: conflict-free rows)

// Flush the top of a wave's per-query histograms (lane = query): bins from the top down until K
// scores are covered.  Dropping lower bins only lowers global counts, so the edge k_hist_tau finds
// stays a valid lower bound; the global top-K scores are all counted, so it stays as tight.
__device__ void flush_hist_top(const uint32_t* hs, int q0, int Q, int K, unsigned int* hist) {
  const int lane = threadIdx.x;
  const int q = q0 + lane;
  if (q >= Q) return;
  const uint32_t* hq = hs + lane * kHRow;
  unsigned int cum = 0;
  for (int w = kBins / 2 - 1; w >= 0 && cum < (unsigned)K; --w) {
    const uint32_t v = hq[w];
    if (v == 0u) continue;
    const unsigned hi = v >> 16, lo = v & 0xFFFFu;  // bins 2w + 1, 2w
    unsigned int* h = hist + (int64_t)q * kBins + 2 * w;
    if (hi) { atomicAdd(h + 1, hi); cum += hi; }
    if (cum < (unsigned)K && lo) { atomicAdd(h, lo); cum += lo; }
  }
}

template <int KS>
__global__ __launch_bounds__(64) void k_sample_hist(SampleArgs a) {
  typedef ZOps<false> Z;
  typedef typename Z::T ZT;
  typedef typename Z::Acc AccT;
  auto zrow = [&](const double* p64, const float*, int64_t row) -> const ZT* { return p64 + row * a.Lp; };
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* hs = reinterpret_cast<uint32_t*>(smem);  // kQW x kHRow words, two u16 counters per word
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.S) c_end = a.S;
  const int q0 = qb * kQW;
  for (int i = lane; i < kQW * kHRow; i += 64) hs[i] = 0u;

  ZT qf[4][KS];
  double qA[4], qB[4], qQ[4], qm[4];
  int qz = 0, qv = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const ZT* zr = zrow(a.Zq, a.Zq32, v ? q : 0) + g * KS;
#pragma unroll
    for (int t = 0; t < KS; ++t) qf[b][t] = v ? zr[t] : (ZT)0;
    const double* st = a.Sq + (int64_t)(v ? q : 0) * a.nseg * 4;
    qm[b] = st[0];
    qA[b] = (0.6 * a.inv_m) * st[1];
    qB[b] = 0.6 * st[0];
    qQ[b] = st[2];
    if (v) qv |= 1 << b;
    if (st[1] == 0.0) qz |= 1 << b;
  }
  __syncthreads();
  typedef double dbl2v __attribute__((ext_vector_type(2)));
  auto load_frag = [&](int64_t cs, ZT* dst) {
    int64_t i = cs + j;
    if (i >= c_end) i = c_end - 1;
    const ZT* p = zrow(a.Zc, a.Zc32, i * a.stride) + g * KS;
#pragma unroll
    for (int t = 0; t < KS; ++t) dst[t] = p[t];
  };
  ZT cf[KS];
  load_frag(c_begin, cf);
  for (int64_t cs = c_begin; cs < c_end; cs += kCS) {
    double cst[12];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int64_t i = cs + Z::row(g, r);
      if (i >= c_end) i = c_end - 1;
      const double* st = a.Sc + i * a.stride * a.nseg * 4;
      const dbl2v v = *reinterpret_cast<const dbl2v*>(st);
      cst[3 * r] = v.x;
      cst[3 * r + 1] = v.y;
      cst[3 * r + 2] = st[2];
    }
    ZT cfn[KS];
    load_frag(cs + kCS, cfn);
    AccT acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = AccT{0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < KS; ++t)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[b] = Z::mfma(cf[t], qf[b][t], acc[b]);  // 4 interleaved chains
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (cs + Z::row(g, r) >= c_end) continue;
      const double cm = cst[3 * r], csd = cst[3 * r + 1], cq = cst[3 * r + 2];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (!((qv >> b) & 1)) continue;
        const bool zq = (qz >> b) & 1, zc = csd == 0.0;
        const double sc = (zq || zc) ? const0(zq, zc, qm[b], cm)
                                     : approx0((double)acc[b][r], a.c1, qA[b], qB[b], qQ[b], csd, cm, cq);
        int bin = (int)(sc * (double)kBins);
        bin = bin < 0 ? 0 : (bin >= kBins ? kBins - 1 : bin);
        atomicAdd(&hs[(16 * b + j) * kHRow + (bin >> 1)], 1u << (16 * (bin & 1)));
      }
    }
#pragma unroll
    for (int t = 0; t < KS; ++t) cf[t] = cfn[t];
  }
  __syncthreads();
  flush_hist_top(hs, q0, a.Q, a.K, a.hist);
}
#endif  // HQ_DIAG

// ------------------------------------------------------------------------------------------------
// Split-f16 level-0 scan (default).  On gfx950 the f32/f64 MFMAs run on the vector ALUs (they never
// co-execute with VALU work: SQ_VALU_MFMA_COEXEC_CYCLES = 0), so the contraction runs on the matrix
// core instead: each normalised value z = hi + lo with hi = f16(z), lo = f16(z - hi), and
//   G ~= hi_q.hi_c + hi_q.lo_c + lo_q.hi_c   (three v_mfma_f32_16x16x32_f16, f32 accumulation)
// for 16 candidates x 16 queries x K = 32 (the level-0 segment zero-padded to 32).  Error budget:
// split and dropped lo.lo <= 3 2^-22 |zq||zc| per term, f32 accumulation of 96 products <= 96 2^-24
// sum|.|, with sum|zq zc| <= m (Cauchy-Schwarz, sum z^2 = m): |dG| <= 2.1e-4 at m = 32; the score
// moves by <= (0.65 / m) |dG| <= 4.3e-6; the f32 epilogue adds < 1e-6 (each term of num is bounded
// by 0.6 rho_q rho_c <= 0.3 den).  The filter passes every pair within kMarginF of the threshold;
// list scores are within ~5.5e-6 of the exact ones (callers re-rank with eps = 2e-5).  Vectors whose
// level-0 statistics are zero-variance or outside [2^-60, 2^60] (f32-unsafe) carry a flag and are
// scored from the f64 statistics.
// ------------------------------------------------------------------------------------------------
constexpr float kMarginF = 6e-5f;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
constexpr int kPad0 = 3 * kCS;  // pad rows of the f32 copies (hq_seg_pack0_split); k_scan0f reads reach cs + 47
// rows of the split statistics S32 (SoA groups of 4 rows, padded)
__host__ __device__ __forceinline__ int64_t pack0_rows(int64_t N) { return ((N + 3) & ~int64_t(3)) + kPad0; }
// Tiled split fragments Z16 (hq_seg_pack0_split): rows in tiles of 16; tile T = [hi: 64 x 8 halves]
// [lo: 64 x 8 halves], the 8 halves at (16 g + j) * 8 holding row 16 T + j, k = 8 g .. 8 g + 7 (the A/B
// operand of lane 16 g + j in v_mfma_f32_16x16x32_f16), so one wave's fragment load is 1 KiB of
// consecutive bytes (16 tag lookups) instead of 16 rows x 64 B (64 lookups).
constexpr int kZ16Tile = 1024;  // halves per 16-row tile
constexpr int kZ16Lo = 512;     // offset of the lo fragments in a tile
__host__ __device__ __forceinline__ int64_t z16_rows(int64_t N) { return ((N + 15) & ~int64_t(15)) + kPad0; }
// the hi fragment (8 halves, k = 8 g .. 8 g + 7) of a row
__host__ __device__ __forceinline__ int64_t z16_frag(int64_t row, int g) {
  return (row >> 4) * kZ16Tile + ((g << 4) + (row & 15)) * 8;
}
// element k (< 32) of a row: hi, and lo at + kZ16Lo
__host__ __device__ __forceinline__ int64_t z16_elem(int64_t row, int k) { return z16_frag(row, k >> 3) + (k & 7); }
// sample rows of the split copies: whole tiles, corpus tile t * stride for sample tile t
__host__ __device__ __forceinline__ int64_t sample_rows_tiled(int64_t N, int64_t stride) {
  return (((N + 15) >> 4) + stride - 1) / stride * 16;
}
__device__ __forceinline__ int64_t sample_row_tiled(int64_t i, int64_t S, int64_t stride) {
  i = i < S ? i : S - 1;
  return (((i >> 4) * stride) << 4) + (i & 15);
}

__device__ __forceinline__ float lower_f32(double x) {  // largest float <= x (x finite or +-inf)
  float f = (float)x;
  if ((double)f > x) {  // step one ulp towards -inf
    const int i = __float_as_int(f);
    f = f > 0.0f ? __int_as_float(i - 1) : (f == 0.0f ? -__int_as_float(1) : __int_as_float(i + 1));
  }
  return f;
}
__device__ __forceinline__ int shr1_f32i(float v) { return shr1_i32(__float_as_int(v)); }

// One wave = 64 queries (4 blocks b of 16: lane (g, j) owns queries 16b + j) x one corpus chunk,
// 16 candidates per step (lane group g owns rows 4g + r, r < 4, of the step: the MFMA D layout).
// Candidate statistics come in the SoA-per-4-rows layout of hq_seg_pack0_split (std[4], mean[4],
// msq[4], flag bits[4] per group of 4 rows), so the filter's packed f32 arithmetic runs over PAIRS OF
// ROWS (r, r+1) of one query: G2 = acc.xy / acc.zw and the statistics pairs are register pairs, the
// query constants are splats — no operand moves.  Per pair:
//   E = base - T = fma(G, c1, 0.35 - T),  num = fma(G, qA cs, qB cm),  d = fma(E, den, num)
//   pass <=> max(E, d) >= 0   (den = msq_q + msq_c >= 0; see filter_half)
// T = thl - kMarginF; 0.35 - T is kept per query (k0) and refreshed only when a threshold moves.
// The step loop is unrolled by two (ping-pong registers for the next step's fragments/statistics),
// candidate pointers advance by a constant per step.
// diagnostics knobs of k_scan0f (HQ_SCAN_EXPT: debug counters, phase skips) exist only in a
// `make DIAG=1` build; the default build compiles them away
#ifdef HQ_DIAG
#define HQ_EXPT(a) ((a).expt)
#else
#define HQ_EXPT(a) 0
#endif

// G-only pre-filter threshold of k_scan0f (see the comment at refresh_k0): smallest G that can pass
// the filter for list threshold t; out of line (rare: called when a threshold moves)
__device__ __noinline__ float gstar0(float t, float qA, float qB, float qQ, float c1f) {
  if (!(t > -__builtin_huge_valf())) return -__builtin_huge_valf();
  if (!(t < __builtin_huge_valf())) return __builtin_huge_valf();
  const double A = qA, B = qB, Qq = qQ, c1 = c1f;
  const double R = ((double)t - (double)kMarginF - 1e-5) - 0.35;
  const double a2 = 4.0 * Qq * c1 * c1 - A * A;
  const double bp = 8.0 * Qq * R * c1;  // the quadratic is a2 G^2 - bp G + c2
  const double c2 = 4.0 * Qq * R * R - B * B;
  double disc = bp * bp - 4.0 * a2 * c2;
  disc = disc > 0.0 ? sqrt(disc) : 0.0;
  const double G = bp >= 0.0 ? (2.0 * c2) / (bp + disc) : (bp - disc) / (2.0 * a2);
  return (float)(G - 1e-6 * (1.0 + fabs(G))) - 1e-5f * (1.0f + fabsf((float)G));
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_scan0f(Scan0Args a) {
  constexpr int NB = 4;
  constexpr int QW = 16 * NB;  // queries per wave
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* ls = reinterpret_cast<float*>(smem);         // QW x K approx scores
  int* li = reinterpret_cast<int*>(ls + QW * a.K);    // QW x K corpus rows
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  // chunks past the corpus end exist when nchunks * chunk_len (both rounded up) exceeds N by more than
  // a chunk (small corpora: N = 3000 -> 192 chunks of 16 rows); their prologue loads (rows c_begin ..
  // c_begin + 31, unclamped) would read past the kPad0 padding rows, so they leave before any load.
  // Every other chunk reads at most row c_end + 46 < N + kPad0.
  if (c_begin >= a.N) return;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.N) c_end = a.N;
  const int q0 = qb * QW;
  const int K = a.K;
  const float c1f = (float)a.c1;
  int cntr[NB] = {};  // pairs offered to the list of query 16b + j (same in the 4 lanes g)

  // queries: fragments, f32 constants, list thresholds (f32, exact list values)
  half8 qh[NB], ql[NB];  // query fragments: k range [8g, 8g + 8) of the hi and lo halves
  float qA[NB], qB[NB], qQ[NB], thl[NB], k0[NB], gs[NB];
  int qsp = 0;  // bit b: query 16b + j is flagged (zero variance / f32-unsafe)
  int qvb = 0;  // bit b: query 16b + j exists
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const int qq = v ? q : 0;
    const _Float16* zr = a.Zq16 + z16_frag(qq, g);
    HQ_GUARD(zr, a.Zq16, z16_rows(a.Q) * 64 - kZ16Lo - 8);
    qh[b] = *reinterpret_cast<const half8*>(zr);
    ql[b] = *reinterpret_cast<const half8*>(zr + kZ16Lo);
    const int64_t gq = (int64_t)(qq >> 2) * 16 + (qq & 3);  // SoA-per-4 statistics
    const float sd = a.Sq32[gq], mn = a.Sq32[gq + 4], ms = a.Sq32[gq + 8];
    const int fl = __float_as_int(a.Sq32[gq + 12]);
    qA[b] = (float)(0.6 * a.inv_m) * sd;
    qB[b] = 0.6f * mn;
    qQ[b] = ms;
    if (v && fl != 0) qsp |= 1 << b;
    if (v) qvb |= 1 << b;
    double t0 = a.thr0;
    if (v && a.th0 && a.th0[q] > t0) t0 = a.th0[q];
    thl[b] = v ? lower_f32(t0) : __builtin_huge_valf();
  }
  // k0 = 0.35 - (thl - margin); flagged queries always pass (+inf), absent ones never (-inf).
  // gs = G-only pre-filter threshold: by Cauchy-Schwarz (num <= sqrt(A^2 G^2 + B^2) sqrt(msq_c)) and
  // AM-GM (den = Q + msq_c >= 2 sqrt(Q msq_c)) every approximate score is at most
  //   U(G) = 0.35 + c1 G + sqrt(A^2 G^2 + B^2) / (2 sqrt(Q))      (A = qA, B = qB, Q = qQ)
  // whatever the candidate; U is strictly increasing (c1 = 0.35/m > A / (2 sqrt Q) <= 0.3/m), so a pair
  // can pass the filter only if G >= G* with U(G*) = T' (T' = thl - margin - 1e-5 slack for the f32
  // evaluation).  G* is the smaller root of 4Q (R - c1 G)^2 = A^2 G^2 + B^2, R = T' - 0.35 (the
  // larger one has R - c1 G < 0), evaluated in f64 and rounded down.
  auto refresh_k0 = [&](const int b) {
    k0[b] = ((qvb >> b) & 1) == 0 ? -__builtin_huge_valf()
                                  : (((qsp >> b) & 1) != 0 ? __builtin_huge_valf() : 0.35f - (thl[b] - kMarginF));
    gs[b] = ((qvb >> b) & 1) == 0 ? __builtin_huge_valf()
                                  : (((qsp >> b) & 1) != 0 ? -__builtin_huge_valf() : gstar0(thl[b], qA[b], qB[b], qQ[b], c1f));
  };
#pragma unroll
  for (int b = 0; b < NB; ++b) refresh_k0(b);
  for (int i = lane; i < QW * K; i += 64) {
    ls[i] = -__builtin_huge_valf();
    li[i] = -1;
  }
  const bool myq = lane < QW && q0 + lane < a.Q;

  // candidate rows are padded (kPad0, hq_seg_pack0_split): no clamping, rows past c_end are masked
  // Candidate statistics: the 16 rows of a step are 4 SoA groups = 64 contiguous floats; lane (g, j)
  // loads float j of group g (one coalesced dword per lane instead of four 16-B loads that 16 lanes
  // repeat), and the values are broadcast within the 16-lane row by DPP row_newbcast when the full
  // filter needs them (rbc<k>).  The flag bits come from one ballot over lanes j >= 12.
  struct CStep {
    half8 f[2];  // fragment: hi, lo of row cs + j, k range [8g, 8g + 8)
    float st;    // SoA statistics float j of group g: std[4], mean[4], msq[4], flags[4]
  };
  struct SStat {
    flt4 sd, mn, ms;  // statistics of rows 4g .. 4g + 3
  };
  const _Float16* pz = a.Zc16 + z16_frag(c_begin + j, g);  // c_begin: a multiple of 16
  const float* pst = a.Sc32 + (c_begin / 4 + g) * 16 + j;
  auto load_step = [&](CStep& c) {
    HQ_GUARD(pz, a.Zc16, z16_rows(a.N) * 64 - kZ16Lo - 8);  // half8 at pz and pz + kZ16Lo
    HQ_GUARD(pst, a.Sc32, pack0_rows(a.N) * 4);
    c.f[0] = *reinterpret_cast<const half8*>(pz);
    c.f[1] = *reinterpret_cast<const half8*>(pz + kZ16Lo);
    c.st = *pst;
    pz += kZ16Tile;
    pst += kCS * 4;
  };
  auto expand = [&](const float st, SStat& x) {
    x.sd = flt4{rbc<0>(st), rbc<1>(st), rbc<2>(st), rbc<3>(st)};
    x.mn = flt4{rbc<4>(st), rbc<5>(st), rbc<6>(st), rbc<7>(st)};
    x.ms = flt4{rbc<8>(st), rbc<9>(st), rbc<10>(st), rbc<11>(st)};
  };
  // bit r: row 4g + r flagged (zero variance / f32-unsafe / pad)
  auto flags = [&](const float st) -> int {
    return (int)(__ballot(j >= 12 && __float_as_int(st) != 0) >> (16 * g + 12)) & 0xF;
  };
  // G of two 16-query blocks: hi.hi + hi.lo + lo.hi, two accumulation chains interleaved
  auto mfma_half = [&](const int h, const half8* f, flt4* acc) {
    acc[0] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
    acc[1] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], qh[2 * h + u], acc[u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], ql[2 * h + u], acc[u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[1], qh[2 * h + u], acc[u], 0, 0, 0);
  };
  // f32 filter of one half; bit 4u + r = pass of pair (query 16(2h+u)+j, row 4g+r).
  // pass <=> base >= T or base + num / den >= T  <=>  max(E, E den + num) >= 0 with E = base - T
  // (den > 0; E den + num is one fma, its sign exact).  Flagged candidates, absent queries and rows
  // past the chunk end are bit masks, applied only when some lane of the wave has a candidate pass
  // (the common half-step ends after one ballot).
  auto filter_half = [&](const int h, const flt4* acc, const float st, const int fm, SStat& x, bool& have,
                         const int rem) -> int {
    // G-only pre-filter (see gstar0): most half-steps end here after 4 max and 2 compares
    const float g0 = fmaxf(fmaxf(acc[0].x, acc[0].y), fmaxf(acc[0].z, acc[0].w));
    const float g1 = fmaxf(fmaxf(acc[1].x, acc[1].y), fmaxf(acc[1].z, acc[1].w));
    const unsigned long long pre = HQ_EXPT(a) == 8 ? 0ull : __ballot((g0 >= gs[2 * h]) | (g1 >= gs[2 * h + 1]) | (fm != 0));
    if (HQ_EXPT(a) == 3 && lane == 0) {
      atomicAdd(a.dbg + 6, 1ull);
      if (pre) atomicAdd(a.dbg + 5, 1ull);
    }
    if (HQ_EXPT(a) != 5 && !pre) return 0;
    if (HQ_EXPT(a) == 7) return 0;  // diagnostics only: base cost of the step (no full filter, no inserts)
    if (!have) {
      expand(st, x);
      have = true;
    }
    const flt2 c1v = {c1f, c1f};
    flt2 m[4];  // [2u + p]: rows (2p, 2p + 1) of query block 2h + u
    float mx = -__builtin_huge_valf();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int b = 2 * h + u;
      const flt2 K0 = {k0[b], k0[b]}, A2 = {qA[b], qA[b]}, B2 = {qB[b], qB[b]}, Q2 = {qQ[b], qQ[b]};
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const flt2 G2 = p == 0 ? acc[u].xy : acc[u].zw;
        const flt2 sd2 = p == 0 ? x.sd.xy : x.sd.zw;
        const flt2 mn2 = p == 0 ? x.mn.xy : x.mn.zw;
        const flt2 ms2 = p == 0 ? x.ms.xy : x.ms.zw;
        const flt2 E = __builtin_elementwise_fma(G2, c1v, K0);
        const flt2 num = __builtin_elementwise_fma(G2, A2 * sd2, B2 * mn2);
        const flt2 d = __builtin_elementwise_fma(E, Q2 + ms2, num);
        const flt2 mm = {fmaxf(E.x, d.x), fmaxf(E.y, d.y)};
        m[2 * u + p] = mm;
        mx = fmaxf(mx, fmaxf(mm.x, mm.y));
      }
    }
    if (!__ballot((mx >= 0.0f) | (fm != 0))) return 0;
    int bits = 0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        bits |= ((int)(m[2 * u + p].x >= 0.0f) << (4 * u + 2 * p)) | ((int)(m[2 * u + p].y >= 0.0f) << (4 * u + 2 * p + 1));
    bits |= fm * 0x11;
    const int nv = rem - 4 * g;  // rows of this lane group inside the chunk
    const int rowm = nv >= 4 ? 0xF : (nv <= 0 ? 0 : (1 << nv) - 1);
    const int b0 = 2 * h, b1 = 2 * h + 1;
    const int qm = (((qvb >> b0) & 1) ? 0x0F : 0) | (((qvb >> b1) & 1) ? 0xF0 : 0);
    return bits & (rowm * 0x11) & qm;
  };
  // List maintenance.  A query's list starts in APPEND mode: passing pairs are appended in parallel
  // (slot from the ballot, no ordering) while the list has room; the pair that fills it sorts it (rank
  // sort), sets the query's threshold to its K-th score and switches it to SORTED mode, where later
  // pairs are merged one at a time.  With the sampled starting thresholds most queries never leave
  // append mode within a chunk.  cntr[b] counts the pairs ever offered (>= K: sorted mode); the slots
  // of a batch follow from its ballot (pairs of query j sit in lanes j, j+16, j+32, j+48).
  auto key_better = [](float s1, int i1, float s2, int i2) { return s1 > s2 || (s1 == s2 && i1 < i2); };
  // rank sort of the first n (<= K <= 64) entries of list qi, in place
  auto sort_list = [&](const int qi, const int n) {
    float e = lane < n ? ls[qi * K + lane] : -__builtin_huge_valf();
    int ei = lane < n ? li[qi * K + lane] : 0x7FFFFFFF;
    int rank = 0;
    for (int o = 0; o < n; ++o) {
      const float so = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), o));
      const int io = __builtin_amdgcn_readlane(ei, o);
      rank += key_better(so, io, e, ei) ? 1 : 0;
    }
    if (lane < n) {
      ls[qi * K + rank] = e;
      li[qi * K + rank] = ei;
    }
  };
  // raise query qi's threshold to tau (lanes holding it) and publish it
  auto raise = [&](const int qi, const float tau) {
    const int b = qi >> 4;
    if (j == (qi & 15)) {
#pragma unroll
      for (int bb = 0; bb < NB; ++bb)
        if (bb == b && tau > thl[bb]) {
          thl[bb] = tau;
          refresh_k0(bb);
        }
    }
    if (lane == 0 && tau > 0.0f) atomicMax(a.gtau + q0 + qi, (unsigned long long)__double_as_longlong((double)tau));
  };
  // merge one pair into the sorted list qi
  auto merge_one = [&](const int qi, const float sc, const int id) {
    float es = lane < K ? ls[qi * K + lane] : -__builtin_huge_valf();
    int ei = lane < K ? li[qi * K + lane] : -1;
    const bool bt = key_better(es, ei, sc, id);
    const int p = __popcll(__ballot(bt));
    if (p >= K) return;
    const float us = __int_as_float(shr1_f32i(es));
    const int ui = shr1_i32(ei);
    if (lane > p) { es = us; ei = ui; }
    if (lane == p) { es = sc; ei = id; }
    if (lane < K) {
      ls[qi * K + lane] = es;
      li[qi * K + lane] = ei;
    }
    raise(qi, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(es), K - 1)));
  };
  // score, test and file the passing pairs of one half: f32 for plain pairs (the filter's expression
  // with the division), f64 statistics for flagged pairs
  auto insert_half = [&](const int h, const flt4* acc, const SStat& c, const int fm, const int64_t cs,
                         const int bits) {
    if (HQ_EXPT(a) == 3 && lane == 0) atomicAdd(a.dbg, 1ull);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 2 * h + u;
        const bool pb = (bits >> (4 * u + r)) & 1;
        const unsigned long long mpb = __ballot(pb);
        if (!mpb) continue;
        if (HQ_EXPT(a) == 3 && lane == 0) {
          atomicAdd(a.dbg + 3, (unsigned long long)__popcll(mpb));
          atomicAdd(a.dbg + 4, 1ull);
        }
        float s = -__builtin_huge_valf();
        const bool flagged = (((qsp >> b) & 1) != 0) | (((fm >> r) & 1) != 0);
        if (pb && !flagged) {
          const float G = acc[u][r];
          const float num = fmaf(G, qA[b] * c.sd[r], qB[b] * c.mn[r]);
          float t = num * __builtin_amdgcn_rcpf(qQ[b] + c.ms[r]);  // 1 ulp
          t = t > 0.0f ? t : 0.0f;
          s = fmaf(G, c1f, 0.35f) + t;
          s = s < 1.0f ? s : 1.0f;
          s = s > 0.0f ? s : 0.0f;
        }
        if (__ballot(pb && flagged)) {
          if (pb && flagged) {
            const int q = q0 + 16 * b + j;
            const double* sq = a.Sq + (int64_t)q * a.nseg * 4;
            const double* sc = a.Sc + (cs + 4 * g + r) * a.nseg * 4;
            HQ_GUARD(sq, a.Sq, (int64_t)a.Q * a.nseg * 4 - 3);
            HQ_GUARD(sc, a.Sc, a.N * a.nseg * 4 - 3);
            const double qm = sq[0], qs = sq[1], qq = sq[2], cm = sc[0], csd = sc[1], cq = sc[2];
            const double v = (qs == 0.0 || csd == 0.0)
                                 ? const0(qs == 0.0, csd == 0.0, qm, cm, (aux_bits(sq) & aux_bits(sc) & kAuxF32) != 0)
                                 : approx0((double)acc[u][r], a.c1, (0.6 * a.inv_m) * qs, 0.6 * qm, qq, csd, cm, cq);
            s = (float)v;
          }
        }
        const bool ok = pb && s >= thl[b];
        const int qi = 16 * b + j;
        const int id = (int)(cs + 4 * g + r);
        const unsigned long long mok = __ballot(ok);
        if (HQ_EXPT(a) == 3 && lane == 0) atomicAdd(a.dbg + 1, (unsigned long long)__popcll(mok));
        const unsigned long long mine = (mok >> j) & 0x0001000100010001ull;  // query j's pairs, bit 16g
        const int pos = cntr[b] + __popcll(mine & ((1ull << (16 * g)) - 1ull));
        cntr[b] += __popcll(mine);
        if (ok && pos < K) {
          ls[qi * K + pos] = s;
          li[qi * K + pos] = id;
        }
        // lists that just filled: sort, threshold
        unsigned long long mf = __ballot(ok && pos == K - 1);
        while (mf) {
          const int l = __builtin_ctzll(mf);
          mf &= mf - 1;
          const int qf = 16 * b + (l & 15);
          sort_list(qf, K);
          raise(qf, ls[qf * K + K - 1]);
        }
        // pairs offered to sorted lists
        unsigned long long mo = __ballot(ok && pos >= K);
        if (HQ_EXPT(a) == 3 && lane == 0) atomicAdd(a.dbg + 2, (unsigned long long)__popcll(mo));
        while (mo) {
          const int l = __builtin_ctzll(mo);
          mo &= mo - 1;
          const float sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), l));
          const int qo = 16 * b + (l & 15);
          if (!(sc >= ls[qo * K + K - 1])) continue;
          merge_one(qo, sc, __builtin_amdgcn_readlane(id, l));
        }
      }
  };

  // Software pipeline: the MFMAs of one half run while the VALU filters the other half
  //   block A: MFMA(step i, half 1)   || filter(step i, half 0)
  //   block B: MFMA(step i+1, half 0) || filter(step i, half 1)
  // Three step buffers: body(i) loads step i + 2 (two bodies of latency cover, the next step's
  // fragments used by this body's second MFMA half were loaded one body earlier)
  CStep cA, cB, cC;
  load_step(cA);
  load_step(cB);
  flt4 acc0[2], acc1[2];
  mfma_half(0, cA.f, acc0);
  unsigned long long gt_bits = 0ull;
  int step = 0;
  auto body = [&](const int64_t cs, const CStep& cur, const CStep& nxt, CStep& nn) {
    load_step(nn);  // rows past the chunk (padded array, kPad0 rows): harmless, masked
    const int rem = (int)(c_end - cs);
    mfma_half(1, cur.f, acc1);
    const int fm = flags(cur.st);
    SStat x;
    bool have = false;
    const int bits0 = filter_half(0, acc0, cur.st, fm, x, have, rem);
    if (__ballot(bits0 != 0)) insert_half(0, acc0, x, fm, cs, bits0);
    mfma_half(0, nxt.f, acc0);
    const int bits1 = filter_half(1, acc1, cur.st, fm, x, have, rem);
    if (__ballot(bits1 != 0)) insert_half(1, acc1, x, fm, cs, bits1);
    if ((step & 3) == 0) {
      if (gt_bits != 0ull) {
        const float gf = (float)__longlong_as_double((long long)gt_bits);  // exact: list values are f32
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float v = __shfl(gf, 16 * b + j, 64);
          if (v > thl[b]) {
            thl[b] = v;
            refresh_k0(b);
          }
        }
      }
      if (myq) gt_bits = __atomic_load_n(a.gtau + q0 + lane, __ATOMIC_RELAXED);
    }
    ++step;
  };
  int64_t cs = c_begin;
  for (; cs + 2 * kCS < c_end; cs += 3 * kCS) {
    body(cs, cA, cB, cC);
    body(cs + kCS, cB, cC, cA);
    body(cs + 2 * kCS, cC, cA, cB);
  }
  if (cs < c_end) body(cs, cA, cB, cC);
  if (cs + kCS < c_end) body(cs + kCS, cB, cC, cA);

  // hand the lists (unordered is fine) to the per-query pools: one atomic per query, lane-parallel
  int nl = 0;  // entries of query `lane`
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int v = __shfl(cntr[b], lane & 15, 64);
    if ((lane >> 4) == b) nl = v < K ? v : K;
  }
  int base = 0;
  if (nl > 0 && myq) base = atomicAdd(a.pool_n + q0 + lane, nl);
  for (int ql = 0; ql < QW; ++ql) {
    const int n = __builtin_amdgcn_readlane(nl, ql);
    if (n == 0 || q0 + ql >= a.Q) continue;
    const int bq = __builtin_amdgcn_readlane(base, ql);
    if (lane < n && bq + lane < a.pool_cap) {  // (pools hold nchunks x k entries for k <= 64: never past)
      const int64_t o = (int64_t)(q0 + ql) * a.pool_cap + bq + lane;
      a.pool_s[o] = ls[ql * K + lane];
      a.pool_i[o] = li[ql * K + lane];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Level-0 scan, queue form (k_scan0g, default since round 3).  Same contraction as k_scan0f (split
// f16, 12 MFMAs per 64 queries x 16 rows) and the same filter and score expressions, reorganised so
// that the per-step vector work fits under the matrix instructions:
//   * no per-wave lists: a pair whose score passes the query's starting threshold (the sampled bound,
//     k_sample_kth, or the caller's threshold) is appended straight to the query's global pool, which
//     k_pool_select reduces to the exact top K (the sample bound admits ~K' x stride pairs per query);
//   * the per-query constants (QConst, computed once per query by k_sample_kth / k_scan_qprep) leave
//     only the G-only pre-filter in the step: two v_max3 and one compare per 16-query block and lane;
//   * a lane block (one query, four rows) passing the pre-filter is appended to a per-wave LDS queue
//     (ballot + mbcnt); the queue is drained 64 entries at a time, one entry per lane: candidate
//     statistics loaded for that entry's four rows, the division-free filter, the f32 score (the f64
//     statistics for flagged rows) and the pool append;
//   * candidate fragments / statistics addressed from a wave-uniform base (scalar step increments).
// Flagged candidate rows (zero variance, f32-unsafe) are skipped by the scan and scored by
// k_pool_select from the f64 statistics before it reads the pools (the corpus's list from hq_seg_flag_rows,
// or k_flag_rows per call; normally none).  Flagged queries
// (zero variance / f32-unsafe) never enter the scan: k_pool_select marks their lists unresolved and the
// caller answers them on the dense exact path.  A pool that would overflow its capacity marks its query
// unresolved the same way.
// ------------------------------------------------------------------------------------------------
struct QConst {
  float qA, qB, qQ, k0;      // 0.6 std / m, 0.6 mean, mean of squares, 0.35 - (thl - margin)
  float thl, gs, low, flag;  // list threshold (f32 lower bound), G* pre-filter bound, 0.1 admitted, query flags
};

// per-query constants of the scan from the query's statistics (std, mean, mean of squares, flag word, as in
// Sq32) and starting threshold t0 (f64)
__device__ __forceinline__ QConst qconst_vals(float sd, float mn, float ms, int fl, double t0, double inv_m) {
  QConst c;
  c.qA = (float)(0.6 * inv_m) * sd;
  c.qB = 0.6f * mn;
  c.qQ = ms;
  c.thl = lower_f32(t0);
  c.flag = __int_as_float(fl);
  if (fl != 0) {  // flagged query: not scanned (dense exact path)
    c.k0 = -__builtin_huge_valf();
    c.gs = __builtin_huge_valf();
    c.low = 0.0f;
  } else {
    c.k0 = 0.35f - (c.thl - kMarginF);
    c.gs = gstar0(c.thl, c.qA, c.qB, c.qQ, (float)(0.35 * inv_m));
    c.low = (0.1f >= c.thl - kMarginF) ? 1.0f : 0.0f;
  }
  return c;
}
__device__ __forceinline__ QConst qconst_of(const float* Sq32, int q, double t0, double inv_m, float c1f) {
  const int64_t gq = (int64_t)(q >> 2) * 16 + (q & 3);  // SoA-per-4 statistics
  (void)c1f;
  return qconst_vals(Sq32[gq], Sq32[gq + 4], Sq32[gq + 8], __float_as_int(Sq32[gq + 12]), t0, inv_m);
}

// one thread per query: QConst from the caller's threshold alone (no sample pass)
__global__ void k_scan_qprep(const float* __restrict__ Sq32, int Q, double thr0, double inv_m,
                             QConst* __restrict__ qc, int* __restrict__ pool_n) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  qc[q] = qconst_of(Sq32, q, thr0, inv_m, 0.0f);
  pool_n[q] = 0;
}

// max of an accumulator in two instructions: IEEE-2019 maximum (v_maximum3_f32 on gfx950; the accumulators
// are never NaN, so it equals fmaxf here).  Compiler-visible, so the MFMA -> VALU read hazard of a fresh
// accumulator gets its wait states from the compiler (fmaxf / fmed3 forms add a v_max canonicalisation of
// each operand in IEEE mode; an inline-asm v_max3 hides the read from the hazard recognizer, the fault
// class of commit ee0b4c1).
__device__ __forceinline__ float max4(const flt4 v) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(v.x, v.y), __builtin_elementwise_maximum(v.z, v.w));
}

constexpr int kQCap = 192;  // LDS queue entries per wave (< 64 before a half-step, which adds at most 128)
// Pool appends staged per wave in LDS: (score, row, query | rank << 8), rank = the entry's position among the
// wave's staged entries of its query; a flush reserves each query's slots with ONE global atomic (lane per
// query) and writes the entries.  Per passing pair, round 4 paid a returning device-scope atomic on the
// query's count: 85 us of a 366 us scan at list length 1008 (diagnostics build, 2M appends on 1000 counters).
constexpr int kStCap = 256;
struct StEntry {
  float s;
  int row, qr;
};
struct QEntry {
  flt4 g;        // G of rows row .. row + 3 for query qi
  int qi, row;   // query within the wave, first row (absolute, multiple of 4)
  int pad0, pad1;
};
// wave-local ordering of the queue's LDS accesses (one wave's LDS instructions execute in issue order;
// this keeps the compiler from moving them across each other)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2v h2(const half8 v, int p) {
  return p == 0 ? __builtin_shufflevector(v, v, 0, 1) : p == 1 ? __builtin_shufflevector(v, v, 2, 3)
       : p == 2 ? __builtin_shufflevector(v, v, 4, 5) : __builtin_shufflevector(v, v, 6, 7);
}

// The split G (hi.hi + hi.lo + lo.hi, f32 accumulation: the three-MFMA contraction, another summation order,
// the same error bound) of query q against rows row0 .. row0 + 3 of the tiled split copies, by v_dot2_f32_f16
// (products exact in f32).  k_scan0g's drain: its pre-filter contracted hi.hi only.
__device__ __forceinline__ flt4 split_g4(const _Float16* __restrict__ Zq16, const _Float16* __restrict__ Zc16, int q,
                                         int64_t row0) {
  flt4 G = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
  for (int gg = 0; gg < 4; ++gg) {  // one k-group at a time: 10 fragment loads in flight, few live VGPRs
    const _Float16* pq = Zq16 + z16_frag(q, gg);
    const half8 qhv = *reinterpret_cast<const half8*>(pq), qlv = *reinterpret_cast<const half8*>(pq + kZ16Lo);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const _Float16* pc = Zc16 + z16_frag(row0 + r, gg);
      const half8 chv = *reinterpret_cast<const half8*>(pc), clv = *reinterpret_cast<const half8*>(pc + kZ16Lo);
      float acc = G[r];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        acc = __builtin_amdgcn_fdot2(h2(qhv, p), h2(chv, p), acc, false);
        acc = __builtin_amdgcn_fdot2(h2(qhv, p), h2(clv, p), acc, false);
        acc = __builtin_amdgcn_fdot2(h2(qlv, p), h2(chv, p), acc, false);
      }
      G[r] = acc;
    }
  }
  return G;
}

// staged pool entries of one wave to the pools (k_scan0g): one count atomic per query with entries, then the
// writes.  Out of line: inlined at every drain site it pushed the scan past 128 VGPRs (spills in the step
// loop); as a call its register saves run only when a flush does (rarely: the stage holds kStCap entries).
__device__ __noinline__ void stage_flush(StEntry* st, int* scnt, int* sbase, int sn, int qw, int q0, int* pool_n,
                                         float* pool_s, int* pool_i, int cap) {
  const int lane = threadIdx.x & 63;
  wave_lds_sync();
  for (int t = lane; t < qw; t += 64) {
    const int c = scnt[t];
    sbase[t] = c > 0 ? atomicAdd(pool_n + q0 + t, c) : 0;
    scnt[t] = 0;
  }
  wave_lds_sync();
  for (int e = lane; e < sn; e += 64) {
    const StEntry x = st[e];
    const int qi = x.qr & 255, slot = sbase[qi] + (x.qr >> 8);
    if (slot < cap) {
      pool_s[(int64_t)(q0 + qi) * cap + slot] = x.s;
      pool_i[(int64_t)(q0 + qi) * cap + slot] = x.row;
    }
  }
  wave_lds_sync();
}

// WPB waves per workgroup: the WPB waves of a block take WPB consecutive query blocks of ONE chunk and
// read the same candidate fragments step by step (a barrier per unrolled iteration keeps them within
// a few steps of each other, so WPB - 1 of the WPB reads of a fragment hit the CU's L1)
// NB 16-query blocks per wave (4: 64 queries; 8: 128 queries, half the corpus fragment loads per MFMA at
// more VGPRs), processed as NB / 2 parts of two blocks, software-pipelined: part p's MFMAs are issued
// before part p - 1's pre-filter reads its accumulators
// HI (default): the pre-filter contracts hi.hi only (one MFMA per 16 x 16 tile instead of three, the corpus
// lo fragments are not loaded): |G_split - G_hihi| <= sum |hq lc| + |lq hc| + f32 accumulation
// < 2^-10 (1.002) m + 1e-5 m, so a lane block passes when max G_hihi >= G* - (1e-3 m + 1e-4); the drain then
// recomputes each queued block's split G (split_g4) for the filter and the pool score.  HI = false: the
// three-MFMA form (option scan_split3).
// OCC: waves per SIMD the register allocation targets (at most 4 since the pool-append stage: 9.7 KB of LDS
// per wave)
template <int WPB, int PF, int NB = 4, bool HI = true, int OCC = 5>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(NB == 8 ? 3 : (HI ? (OCC < 4 ? OCC : 4) : 1)))) void k_scan0g(Scan0Args a) {
  constexpr int QW = 16 * NB, NP = NB / 2;
  using QE = QEntry;  // G_hh kept for the drain's gate (QEntryHI: no gate, measured slower)
  __shared__ QE qe_all[WPB][kQCap];
  __shared__ StEntry st_all[WPB][kStCap];
  __shared__ int scnt_all[WPB][QW], sbase_all[WPB][QW];
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  QE* qe = qe_all[WPB > 1 ? threadIdx.x >> 6 : 0];
  StEntry* st = st_all[WPB > 1 ? threadIdx.x >> 6 : 0];
  int* scnt = scnt_all[WPB > 1 ? threadIdx.x >> 6 : 0];
  int* sbase = sbase_all[WPB > 1 ? threadIdx.x >> 6 : 0];
  for (int t = lane; t < QW; t += 64) scnt[t] = 0;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int nqg = (a.nqb + WPB - 1) / WPB;
  const int chunk = xcd + 8 * (slot / nqg);
  const int qb = (slot % nqg) * WPB + (WPB > 1 ? (int)(threadIdx.x >> 6) : 0);
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  if (c_begin >= a.N) return;  // chunks past the corpus end (k_scan0f comment)
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.N) c_end = a.N;
  const int q0 = qb * QW;
  const float c1f = (float)a.c1;
  const QConst* qc = reinterpret_cast<const QConst*>(a.qconst);

  half8 qh[NB], ql[HI ? 1 : NB];
  float gs[NB];
  const float dG = HI ? (float)(1e-3 / a.inv_m) + 1e-4f : 0.0f;  // hi.hi pre-filter slack (above)
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const int qq = v ? q : 0;
    const _Float16* zr = a.Zq16 + z16_frag(qq, g);
    HQ_GUARD(zr, a.Zq16, z16_rows(a.Q) * 64 - kZ16Lo - 8);
    qh[b] = *reinterpret_cast<const half8*>(zr);
    if constexpr (!HI) ql[b] = *reinterpret_cast<const half8*>(zr + kZ16Lo);
    gs[b] = v ? qc[q].gs - dG : __builtin_huge_valf();
  }

  // wave-uniform bases, per-lane constant offsets (scalar step increments)
  const char* zb = reinterpret_cast<const char*>(a.Zc16 + (c_begin >> 4) * kZ16Tile);  // c_begin: a multiple of 16
  const int zoff = lane * 16;  // bytes: the lane's 8 halves of a tile
  struct CStep {
    half8 f[HI ? 1 : 2];
  };
#ifdef HQ_DIAG
  const int64_t smul = (a.expt == 5 || a.expt == 6) ? 0 : kZ16Tile * 2;  // timing experiments: step 0 only
#else
  constexpr int64_t smul = kZ16Tile * 2;
#endif
  auto load_step = [&](CStep& c, const int64_t s) {
    const _Float16* p = reinterpret_cast<const _Float16*>(zb + s * smul + zoff);
    HQ_GUARD(p, a.Zc16, z16_rows(a.N) * 64 - kZ16Lo - 8);
    c.f[0] = *reinterpret_cast<const half8*>(p);
    if constexpr (!HI) c.f[HI ? 0 : 1] = *reinterpret_cast<const half8*>(p + kZ16Lo);
  };
  auto mfma_part = [&](const int h, const half8* f, flt4* acc) {
    acc[0] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
    acc[1] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], qh[2 * h + u], acc[u], 0, 0, 0);
    if constexpr (!HI) {
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], ql[2 * h + u], acc[u], 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 2; ++u)
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[HI ? 0 : 1], qh[2 * h + u], acc[u], 0, 0, 0);
    }
  };

  int qn = 0;  // queue entries (wave-uniform)
  int sn = 0;  // staged pool entries (wave-uniform)
  auto flush = [&]() {
    stage_flush(st, scnt, sbase, sn, QW, q0, a.pool_n, a.pool_s, a.pool_i, a.pool_cap);
    sn = 0;
  };
  // drain n <= 64 entries from the front of the queue, then shift the rest down
  auto drain = [&](const int n) {
    if (lane < n) {
      float sc[4] = {-1.0f, -1.0f, -1.0f, -1.0f};  // pool scores of the entry's rows (< 0: not appended)
      const int eqi = qe[lane].qi, erow = qe[lane].row;
      const int q = q0 + eqi;
      flt4 eg = qe[lane].g;
      const QConst c = qc[q];
      const float* stt = a.Sc32 + (int64_t)(erow >> 2) * 16;  // the SoA group of rows row .. row + 3
      HQ_GUARD(stt, a.Sc32, pack0_rows(a.N) * 4 - 15);
      const flt4 sd = *reinterpret_cast<const flt4*>(stt);
      const flt4 mn = *reinterpret_cast<const flt4*>(stt + 4);
      const flt4 ms = *reinterpret_cast<const flt4*>(stt + 8);
      const flt4 fl = *reinterpret_cast<const flt4*>(stt + 12);
      bool need = true;
      if constexpr (HI) {
        // gate: the filter is monotone in G and G_split <= G_hh + dG, so a block none of whose rows passes at
        // G_hh + dG needs no split recompute (most queued blocks: the G-only pre-filter is looser)
        need = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float Gu = eg[r] + dG;
          const float E = fmaf(Gu, c1f, c.k0);
          const float d = fmaf(E, c.qQ + ms[r], fmaf(Gu, c.qA * sd[r], c.qB * mn[r]));
          need |= erow + r < c_end && __float_as_int(fl[r]) == 0 && fmaxf(E, d) >= 0.0f;
        }
        if (need) eg = split_g4(a.Zq16, a.Zc16, q, erow);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = erow + r;
        const int f = __float_as_int(fl[r]);
        if (!need || row >= c_end || f != 0) continue;  // past the chunk; flagged rows: k_pool_select
        const float G = eg[r];
        // division-free filter (k_scan0f filter_half), then the list score (k_scan0f insert_half)
        const float E = fmaf(G, c1f, c.k0);
        const float num = fmaf(G, c.qA * sd[r], c.qB * mn[r]);
        const float d = fmaf(E, c.qQ + ms[r], num);
        if (fmaxf(E, d) >= 0.0f) {
          float t = num * __builtin_amdgcn_rcpf(c.qQ + ms[r]);
          t = t > 0.0f ? t : 0.0f;
          float v = fmaf(G, c1f, 0.35f) + t;
          v = v < 1.0f ? v : 1.0f;
          v = v > 0.0f ? v : 0.0f;
          if (v >= c.thl) sc[r] = v;
        }
      }
      qe[lane].g = flt4{sc[0], sc[1], sc[2], sc[3]};  // the entry's pool scores replace its G (consumed)
    }
    wave_lds_sync();
    // stage the passing rows: ballot + mbcnt positions, LDS ranks per query (one flush check per drain)
    const flt4 ps = lane < n ? qe[lane].g : flt4{-1.0f, -1.0f, -1.0f, -1.0f};
    unsigned long long pm[4];
    int call = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pm[r] = __builtin_amdgcn_ballot_w64(ps[r] >= 0.0f);
      call += __popcll(pm[r]);
    }
    if (call > 0) {
      if (sn + call > kStCap) flush();
      const int eqi = lane < n ? qe[lane].qi : 0, erow = lane < n ? qe[lane].row : 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (ps[r] >= 0.0f) {
          const int rank = atomicAdd(&scnt[eqi], 1);
          const unsigned long long m = pm[r];
          const int e = sn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
          st[e] = StEntry{ps[r], erow + r, eqi | (rank << 8)};
        }
        sn += __popcll(pm[r]);
      }
    }
    wave_lds_sync();
    // shift the remaining entries down (all reads of a 64-entry block before its writes)
    for (int b0 = n; b0 < qn; b0 += 64) {
      const bool mv = b0 + lane < qn;
      flt4 tg = {0.0f, 0.0f, 0.0f, 0.0f};
      int tq = 0, tr = 0;
      if (mv) {
        tg = qe[b0 + lane].g;
        tq = qe[b0 + lane].qi;
        tr = qe[b0 + lane].row;
      }
      wave_lds_sync();
      if (mv) {
        qe[b0 - n + lane].g = tg;
        qe[b0 - n + lane].qi = tq;
        qe[b0 - n + lane].row = tr;
      }
      wave_lds_sync();
    }
    qn -= n;
  };
  // enqueue the lane blocks of one part whose pre-filter passed (masks m0, m1: blocks 2h, 2h + 1)
  auto enqueue = [&](const int h, const flt4* acc, const unsigned long long m0, const unsigned long long m1,
                     const int64_t cs) {
    const int c0 = __popcll(m0);
    const unsigned lo0 = __builtin_amdgcn_mbcnt_lo((unsigned)m0, 0u), lo1 = __builtin_amdgcn_mbcnt_lo((unsigned)m1, 0u);
    if ((m0 >> lane) & 1ull) {
      const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), lo0);
      qe[pos].g = acc[0];
      qe[pos].qi = 32 * h + j;
      qe[pos].row = (int)(cs + 4 * g);
    }
    if ((m1 >> lane) & 1ull) {
      const int pos = qn + c0 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), lo1);
      qe[pos].g = acc[1];
      qe[pos].qi = 32 * h + 16 + j;
      qe[pos].row = (int)(cs + 4 * g);
    }
    qn += c0 + __popcll(m1);
  };
  // pre-filter of one half: max of the lane's four rows per block against G* (the compare's lane mask
  // is the ballot); blocks holding a flagged row (f32-unsafe; zero-variance for a query that admits 0.1)
  // are queued regardless
#ifdef HQ_DIAG
  if (a.expt == 6)  // timing experiment: nothing is queued
    for (int b = 0; b < NB; ++b) gs[b] = __builtin_huge_valf();
#endif
  auto part_step = [&](const int h, const flt4* acc, const int64_t cs) {
    const unsigned long long m0 = __builtin_amdgcn_ballot_w64(max4(acc[0]) >= gs[2 * h]);
    const unsigned long long m1 = __builtin_amdgcn_ballot_w64(max4(acc[1]) >= gs[2 * h + 1]);
    if (m0 | m1) {
      enqueue(h, acc, m0, m1, cs);
      while (qn >= 64) drain(64);  // keeps qn < 64 before each half-step: the queue never exceeds 191
    }
  };

  // PF + 1 step buffers in rotation: the fragments of step s + PF are requested while step s is computed
  // (the prefetch index is clamped to the chunk's last step: no read past its rows + 15)
  const int64_t nsteps = (c_end - c_begin + kCS - 1) / kCS;
  CStep buf[PF + 1];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_step(buf[u], u < nsteps ? u : nsteps - 1);
  flt4 acc[NP][2];
  mfma_part(0, buf[0].f, acc[0]);
#ifdef HQ_DIAG
  // timing experiments: 7 = no pre-filter (loads + MFMAs only), 9 = no loads after the prologue
  const bool x_nofilter = a.expt == 7, x_noload = a.expt == 9;
#else
  constexpr bool x_nofilter = false, x_noload = false;
#endif
  auto body = [&](const int64_t s, const CStep& cur, const CStep& nxt, CStep& nn) {
    if (!x_noload) load_step(nn, s + PF < nsteps ? s + PF : nsteps - 1);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch PF steps ahead (the scheduler sinks it otherwise)
    const int64_t cs = c_begin + s * kCS;
#pragma unroll
    for (int p = 1; p < NP; ++p) {
      mfma_part(p, cur.f, acc[p]);
      if (!x_nofilter) part_step(p - 1, acc[p - 1], cs);
    }
    mfma_part(0, nxt.f, acc[0]);
    if (!x_nofilter) part_step(NP - 1, acc[NP - 1], cs);
  };
  int64_t s = 0;
  for (; s + PF < nsteps; s += PF + 1) {
#pragma unroll
    for (int u = 0; u <= PF; ++u) body(s + u, buf[u], buf[(u + 1) % (PF + 1)], buf[(u + PF) % (PF + 1)]);
    if constexpr (WPB > 1) __builtin_amdgcn_s_barrier();  // same step count in every wave of the block
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (s + u < nsteps) body(s + u, buf[u], buf[(u + 1) % (PF + 1)], buf[(u + PF) % (PF + 1)]);
  while (qn > 0) drain(qn < 64 ? qn : 64);
  if (sn > 0) flush();
}

// rows of the split copies with a zero-variance / f32-unsafe flag (S32 flag word bits 1, 2): compacted
// into list[*count] (order irrelevant: the pools are selected by (score, row))
__global__ __launch_bounds__(256) void k_flag_rows(const float* __restrict__ S32, int64_t N, int* __restrict__ list,
                                                   int* __restrict__ count) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
    const int f = __float_as_int(S32[(r >> 2) * 16 + 12 + (r & 3)]);
    if (f & 3) list[atomicAdd(count, 1)] = (int)r;
  }
}

// one flagged row against one scanned query: the f64 statistics as k_scan0f's insert
// path (const0 for zero variance, approx0 with G from the split copies otherwise), appended to the pools
// when the score reaches the query's list threshold
__device__ __forceinline__ void flagged_pair(const Scan0Args& a, const QConst& c, int q, int row) {
  const double* sq = a.Sq + (int64_t)q * a.nseg * 4;
  const _Float16* zq = a.Zq16;
  const double* sc = a.Sc + (int64_t)row * a.nseg * 4;
  const double qm = sq[0], qs = sq[1], qq = sq[2], cm = sc[0], csd = sc[1], cq = sc[2];
  double v;
  if (qs == 0.0 || csd == 0.0) {
    v = const0(qs == 0.0, csd == 0.0, qm, cm, (aux_bits(sq) & aux_bits(sc) & kAuxF32) != 0);
  } else {
    const _Float16* zc = a.Zc16;
    double G = 0.0;
    for (int k = 0; k < 32; ++k) {
      const int64_t eq = z16_elem(q, k), ec = z16_elem(row, k);
      G = fma((double)zq[eq] + (double)zq[eq + kZ16Lo], (double)zc[ec] + (double)zc[ec + kZ16Lo], G);
    }
    v = approx0(G, a.c1, (0.6 * a.inv_m) * qs, 0.6 * qm, qq, csd, cm, cq);
  }
  const float sv = (float)v;
  if (sv >= c.thl) {
    const int slot = atomicAdd(a.pool_n + q, 1);
    if (slot < a.pool_cap) {
      a.pool_s[(int64_t)q * a.pool_cap + slot] = sv;
      a.pool_i[(int64_t)q * a.pool_cap + slot] = row;
    }
  }
}

// Exact top-K of each query's pool (one wave per query): (score desc, row asc).  The K-th largest
// score v is found by bisection on the f32 bit pattern (scores >= 0), ties at v by bisection on the
// row, then the K selected entries are rank-sorted.  Pools of up to 64*kPoolReg entries stay in
// registers; larger ones are re-read per bisection step.
constexpr int kPoolReg = 16;

// th0 / thr0: the scan's sampled starting thresholds and the caller's threshold.  A starting threshold
// from the sample's K'-th best (K' < K, see k_sample_kth) is not a provable lower bound of the K-th
// best: a query whose pool then holds fewer than K entries while th0 > thr0 may miss pairs below th0,
// so its empty slots are marked with score +inf (id -1), which hq_refine_topk reads as "unresolved".
// pool_s / pool_i / pool_n are plain pointers (no const, no __restrict__): flagged_pair appends to the same
// pools through fa.pool_* before they are read
__global__ __launch_bounds__(64) void k_pool_select(float* pool_s, int* pool_i, int* pool_n, int cap, int Q, int K,
                                                    int64_t id_base, double* __restrict__ out_score,
                                                    int64_t* __restrict__ out_id, const double* __restrict__ th0,
                                                    double thr0, const float* __restrict__ qflag, int qstride,
                                                    Scan0Args fa, const int* __restrict__ flist,
                                                    const int* __restrict__ fcount) {
  const int lane = threadIdx.x;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    // fcount != null (k_scan0g): the corpus's flagged rows against this query first (lanes over the
    // rows), appended to the pool before it is read; pool_n is then read with an
    // L1-bypassing load (the appends are L2 atomics)
    // the flagged-row count, the pool count and the query's flag word are requested together (one round
    // trip; the pool count is read again after flagged appends, which are rare)
    const int nfl = fcount ? *fcount : 0;
    int pn = fcount ? __hip_atomic_load(pool_n + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pool_n[q];
    const int qfw = qflag ? __float_as_int(qflag[(int64_t)q * qstride]) : 0;
    if (fcount) {
      const QConst* qc = reinterpret_cast<const QConst*>(fa.qconst);
      const bool app = nfl > 0 && __float_as_int(qc[q].flag) == 0;
      if (app) {
        const QConst c = qc[q];
        for (int i = lane; i < nfl; i += 64) flagged_pair(fa, c, q, flist[i]);
      }
      __syncthreads();
      if (app) pn = __hip_atomic_load(pool_n + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // k_scan0g / k_scanov (qflag: the query's flag word in its constants, qstride floats apart): a flagged
    // query (not scanned) or an overflowing pool -> every slot +inf / -1, which the exact re-rank reads
    // as unresolved (the caller's dense exact path answers the query)
    if (qflag && (qfw != 0 || pn > cap)) {
      for (int x = lane; x < K; x += 64) {
        out_score[(int64_t)q * K + x] = __builtin_huge_val();
        out_id[(int64_t)q * K + x] = -1;
      }
      continue;
    }
#ifdef HQ_DIAG
    const int T = (int)diag_bound(pn, (int64_t)cap + 1, __LINE__);
#else
    const int T = pn;
#endif
    const float* ps = pool_s + (int64_t)q * cap;
    const int* pi = pool_i + (int64_t)q * cap;
    const bool inreg = T <= 64 * kPoolReg;
    float rs[kPoolReg];
    int ri[kPoolReg];
    if (inreg) {
#pragma unroll
      for (int e = 0; e < kPoolReg; ++e) {
        const int x = lane + 64 * e;
        rs[e] = x < T ? ps[x] : -1.0f;
        ri[e] = x < T ? pi[x] : 0x7FFFFFFF;
      }
    }
    // count entries with (score > sv) or (score == sv and row <= iv)  [iv = -1: score > sv only;
    // iv = INT_MAX: score >= sv]
    auto count = [&](float sv, int iv) -> int {
      int c = 0;
      if (inreg) {
#pragma unroll
        for (int e = 0; e < kPoolReg; ++e) c += (rs[e] > sv || (rs[e] == sv && ri[e] <= iv)) ? 1 : 0;
      } else {
        for (int x = lane; x < T; x += 64) {
          const float s = ps[x];
          c += (s > sv || (s == sv && pi[x] <= iv)) ? 1 : 0;
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
      return c;
    };
    const int k = T < K ? T : K;
    // Fast path (pool in registers, > K entries): T0 = the K-th largest lane maximum.  At least K
    // entries are >= T0 (those K maxima), so the top K all are; when at most 64 entries are >= T0
    // (the common case) they are gathered and rank-sorted directly, without the bisection.
    if (inreg && T > K) {
      float lm = -1.0f;
#pragma unroll
      for (int e = 0; e < kPoolReg; ++e) lm = rs[e] > lm ? rs[e] : lm;
      int lr = 0;  // rank of this lane's maximum (value desc, lane asc)
      for (int o = 0; o < 64; ++o) {
        const float mo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lm), o));
        lr += (mo > lm || (mo == lm && o < lane)) ? 1 : 0;
      }
      const unsigned long long mk = __ballot(lr == K - 1);
      const float t0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lm), __builtin_ctzll(mk)));
      __shared__ float fs[64];
      __shared__ int fi[64];
      int c = 0;
#pragma unroll
      for (int e = 0; e < kPoolReg; ++e) {
        const bool sel = rs[e] >= t0 && lane + 64 * e < T;
        const unsigned long long m = __ballot(sel);
        const int pre = c + __popcll(m & ((1ull << lane) - 1ull));
        if (sel && pre < 64) { fs[pre] = rs[e]; fi[pre] = ri[e]; }
        c += __popcll(m);
      }
      if (c <= 64) {
        __syncthreads();
        const float es = lane < c ? fs[lane] : -1.0f;
        const int ei = lane < c ? fi[lane] : 0x7FFFFFFF;
        int rank = 0;
        for (int o = 0; o < c; ++o) {
          const float so = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(es), o));
          const int io = __builtin_amdgcn_readlane(ei, o);
          rank += (so > es || (so == es && io < ei)) ? 1 : 0;
        }
        if (lane < c && rank < K) {
          out_score[(int64_t)q * K + rank] = (double)es;
          out_id[(int64_t)q * K + rank] = (int64_t)ei + id_base;
        }
        __syncthreads();
        continue;
      }
      __syncthreads();
    }
    float sv = -1.0f;
    int iv = 0x7FFFFFFF;  // select all
    if (T > K) {
      // largest sv (as bits) with count(score >= sv) >= K
      unsigned lo = 0, hi = 0x7F800000u;  // [0, +inf]
      while (lo < hi) {
        const unsigned mid = lo + (hi - lo + 1) / 2;
        if (count(__uint_as_float(mid), 0x7FFFFFFF) >= K) lo = mid; else hi = mid - 1;
      }
      sv = __uint_as_float(lo);
      const int gt = count(sv, -1);  // strictly above sv
      // smallest iv with count(score > sv or (== sv and row <= iv)) >= K
      int a0 = 0, a1 = 0x7FFFFFFE;
      if (gt < K) {
        while (a0 < a1) {
          const int mid = a0 + (a1 - a0) / 2;
          if (count(sv, mid) >= K) a1 = mid; else a0 = mid + 1;
        }
      }
      iv = gt < K ? a0 : -1;
    }
    // gather the k selected entries (rank among the selected by ballot prefix), then rank-sort
    __shared__ float gs[64];
    __shared__ int gi[64];
    int filled = 0;
    auto consider = [&](float s, int id, bool valid) {
      const bool sel = valid && (s > sv || (s == sv && id <= iv));
      const unsigned long long m = __ballot(sel);
      const int pre = __popcll(m & ((1ull << lane) - 1ull));
      if (sel && filled + pre < 64) { gs[filled + pre] = s; gi[filled + pre] = id; }
      filled += __popcll(m);
    };
    if (inreg) {
#pragma unroll
      for (int e = 0; e < kPoolReg; ++e) consider(rs[e], ri[e], lane + 64 * e < T);
    } else {
      for (int x0 = 0; x0 < T; x0 += 64) {
        const int x = x0 + lane;
        consider(x < T ? ps[x] : -1.0f, x < T ? pi[x] : 0, x < T);
      }
    }
    __syncthreads();
    const float es = lane < k ? gs[lane] : -1.0f;
    const int ei = lane < k ? gi[lane] : 0x7FFFFFFF;
    int rank = 0;
    for (int o = 0; o < k; ++o) {
      const float so = __shfl(es, o, 64);
      const int io = __shfl(ei, o, 64);
      rank += (so > es || (so == es && io < ei)) ? 1 : 0;
    }
    if (lane < k) {
      out_score[(int64_t)q * K + rank] = (double)es;
      out_id[(int64_t)q * K + rank] = (int64_t)ei + id_base;
    }
    if (lane >= k && lane < K) {
      const bool trunc = th0 != nullptr && th0[q] > thr0;
      out_score[(int64_t)q * K + lane] = trunc ? __builtin_huge_val() : -__builtin_huge_val();
      out_id[(int64_t)q * K + lane] = -1;
    }
    __syncthreads();
  }
}

#ifdef HQ_DIAG
// f32 sample pass: f32 scores of a strided subset into per-query histograms; flagged pairs are not
// counted (which only lowers the bound)
__global__ __launch_bounds__(64) void k_sample_histf(SampleArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* hs = reinterpret_cast<uint32_t*>(smem);  // kQW x kHRow words, two u16 counters per word
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.S) c_end = a.S;
  const int q0 = qb * kQW;
  const float c1f = (float)a.c1;
  for (int i = lane; i < kQW * kHRow; i += 64) hs[i] = 0u;

  half8 qh[4], ql[4];
  float qA[4], qB[4], qQ[4];
  int qok = 0;  // bit b: valid, unflagged query
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const int qq = v ? q : 0;
    const _Float16* zr = a.Zq16 + z16_frag(qq, g);
    qh[b] = *reinterpret_cast<const half8*>(zr);
    ql[b] = *reinterpret_cast<const half8*>(zr + kZ16Lo);
    const int64_t gq = (int64_t)(qq >> 2) * 16 + (qq & 3);  // SoA-per-4 statistics
    qA[b] = (float)(0.6 * a.inv_m) * a.Sq32[gq];
    qB[b] = 0.6f * a.Sq32[gq + 4];
    qQ[b] = a.Sq32[gq + 8];
    if (v && __float_as_int(a.Sq32[gq + 12]) == 0) qok |= 1 << b;
  }
  __syncthreads();
  auto row_of = [&](int64_t i) -> int64_t { return sample_row_tiled(i, a.S, a.stride); };
  auto load_frag = [&](int64_t cs, half8* dst) {
    const _Float16* p = a.Zc16 + z16_frag(row_of(cs + j), g);
    HQ_GUARD(p, a.Zc16, z16_rows(a.N) * 64 - kZ16Lo - 8);
    dst[0] = *reinterpret_cast<const half8*>(p);
    dst[1] = *reinterpret_cast<const half8*>(p + kZ16Lo);
  };
  half8 cf[2];
  load_frag(c_begin, cf);
  float cut[4] = {-1.0f, -1.0f, -1.0f, -1.0f};  // per query: scores below need no counting
  int step = 0;
  for (int64_t cs = c_begin; cs < c_end; cs += kCS) {
    flt4 cst[4];  // (std, mean, msq, flags) of rows 4g + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = row_of(cs + 4 * g + r);
      const float* p = a.Sc32 + (row >> 2) * 16 + (row & 3);
      cst[r] = flt4{p[0], p[4], p[8], p[12]};
    }
    half8 cfn[2];
    load_frag(cs + kCS, cfn);
    flt4 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], qh[b], flt4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], ql[b], acc[b], 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[1], qh[b], acc[b], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = cs + 4 * g + r < c_end && __float_as_int(cst[r].w) == 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float G = acc[b][r];
        // division-free test against the cut first (most pairs stop here)
        const float R = cut[b] - fmaf(G, c1f, 0.35f);
        const float num = fmaf(G, qA[b] * cst[r].x, qB[b] * cst[r].y);
        const float den = qQ[b] + cst[r].z;
        if (!ok || !((qok >> b) & 1) || !((R <= 0.0f) || (num >= R * den))) continue;
        float t = num * __builtin_amdgcn_rcpf(den);
        t = t > 0.0f ? t : 0.0f;
        const float sc = fmaf(G, c1f, 0.35f) + t;
        int bin = (int)(sc * (float)kBins);
        bin = bin < 0 ? 0 : (bin >= kBins ? kBins - 1 : bin);
        atomicAdd(&hs[(16 * b + j) * kHRow + (bin >> 1)], 1u << (16 * (bin & 1)));
      }
    }
    cf[0] = cfn[0];
    cf[1] = cfn[1];
    // every 8 steps: cut = lower edge of the bin holding this wave's K-th best score of each query;
    // lower bins would never be flushed (flush_hist_top stops at K), so they need not be counted
    if ((++step & 7) == 0) {
      const uint32_t* hq = hs + lane * kHRow;
      unsigned int cum = 0;
      int e = -1;
      for (int w = kBins / 2 - 1; w >= 0; --w) {
        const uint32_t v = hq[w];
        cum += v >> 16;
        if (cum >= (unsigned)a.K) { e = 2 * w + 1; break; }
        cum += v & 0xFFFFu;
        if (cum >= (unsigned)a.K) { e = 2 * w; break; }
      }
      const float cv = e > 0 ? (float)e / (float)kBins - 1e-6f : -1.0f;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float v = __shfl(cv, 16 * b + j, 64);
        cut[b] = v > cut[b] ? v : cut[b];
      }
    }
  }
  __syncthreads();
  flush_hist_top(hs, q0, a.Q, a.K, a.hist);
}
#endif  // HQ_DIAG

// f32 sample pass, top-T form (default): no histogram.  Every lane (g, j) keeps, for each of its
// four queries 16b + j, the kTopT best approximate scores of its own stream of sample rows (rows 4g ..
// 4g + 3 of every step of its chunk), tested division-free against its own kTopT-th best.  The values
// of all streams are real scores of distinct (query, row) pairs, so the K-th best of their union
// (k_sample_kth) is a lower bound of the K-th best over the sample and hence over the corpus; it is
// as tight as the sample's own K-th unless a stream held more than kTopT of the sample's top K.
// No LDS, no atomics: occupancy is set by VGPRs alone.  Output: top[(q * nstreams + 4 chunk + g) *
// kTopT + t], every entry of every existing query written (-1 = empty).
constexpr int kTopT = 2;

__global__ __launch_bounds__(64) void k_sample_topf(SampleArgs a) {
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.S) c_end = a.S;
  const int q0 = qb * kQW;
  const float c1f = (float)a.c1;

  half8 qh[4], ql[4];
  float qA[4], qB[4], qQ[4];
  int qok = 0;  // bit b: valid, unflagged query
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const int qq = v ? q : 0;
    const _Float16* zr = a.Zq16 + z16_frag(qq, g);
    qh[b] = *reinterpret_cast<const half8*>(zr);
    ql[b] = *reinterpret_cast<const half8*>(zr + kZ16Lo);
    const int64_t gq = (int64_t)(qq >> 2) * 16 + (qq & 3);  // SoA-per-4 statistics
    qA[b] = (float)(0.6 * a.inv_m) * a.Sq32[gq];
    qB[b] = 0.6f * a.Sq32[gq + 4];
    qQ[b] = a.Sq32[gq + 8];
    if (v && __float_as_int(a.Sq32[gq + 12]) == 0) qok |= 1 << b;
  }
  float top[4][kTopT];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int t = 0; t < kTopT; ++t) top[b][t] = -1.0f;
  // k0[b] = 0.35 - (current kTopT-th best); +inf-free: an invalid / flagged query never passes
  float k0[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) k0[b] = ((qok >> b) & 1) ? 1.35f : -__builtin_huge_valf();
  auto row_of = [&](int64_t i) -> int64_t { return sample_row_tiled(i, a.S, a.stride); };
  auto load_frag = [&](int64_t cs, half8* dst) {
    const _Float16* p = a.Zc16 + z16_frag(row_of(cs + j), g);
    HQ_GUARD(p, a.Zc16, z16_rows(a.N) * 64 - kZ16Lo - 8);
    dst[0] = *reinterpret_cast<const half8*>(p);
    dst[1] = *reinterpret_cast<const half8*>(p + kZ16Lo);
  };
  // statistics: lane (g, j) loads stat (j & 3) (std, mean, msq, flags) of row 4g + (j >> 2) - one dword
  // per lane - and the 16 values of the lane group are broadcast by DPP row_newbcast
  auto load_stats = [&](int64_t cs) -> float {
    const int64_t row = row_of(cs + 4 * g + (j >> 2));
    const float* p = a.Sc32 + (row >> 2) * 16 + (j & 3) * 4 + (row & 3);
    HQ_GUARD(p, a.Sc32, pack0_rows(a.N) * 4);  // sample tiles may end in pad rows (flag 4: not scored)
    return *p;
  };
  // fragments and statistics are loaded two steps ahead (3-buffer rotation, as in k_scan0f): at 2 waves
  // per SIMD one step of strided-row latency was exposed per step
  half8 cf[2], cf1[2];
  load_frag(c_begin, cf);
  float stv = load_stats(c_begin);
  load_frag(c_begin + kCS, cf1);
  float st1 = load_stats(c_begin + kCS);
  for (int64_t cs = c_begin; cs < c_end; cs += kCS) {
    half8 cfn[2];
    load_frag(cs + 2 * kCS, cfn);
    const float stn = load_stats(cs + 2 * kCS);
    const flt4 cst[4] = {flt4{rbc<0>(stv), rbc<1>(stv), rbc<2>(stv), rbc<3>(stv)},
                         flt4{rbc<4>(stv), rbc<5>(stv), rbc<6>(stv), rbc<7>(stv)},
                         flt4{rbc<8>(stv), rbc<9>(stv), rbc<10>(stv), rbc<11>(stv)},
                         flt4{rbc<12>(stv), rbc<13>(stv), rbc<14>(stv), rbc<15>(stv)}};
    flt4 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], qh[b], flt4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], ql[b], acc[b], 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[1], qh[b], acc[b], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    // division-free test against the lane's own kTopT-th best: score > t <=> max(E, E den + num) > 0
    int bits = 0;  // bit 4b + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = cs + 4 * g + r < c_end && __float_as_int(cst[r].w) == 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float G = acc[b][r];
        const float E = fmaf(G, c1f, k0[b]);
        const float num = fmaf(G, qA[b] * cst[r].x, qB[b] * cst[r].y);
        const float d = fmaf(E, qQ[b] + cst[r].z, num);
        bits |= (int)(ok && fmaxf(E, d) > 0.0f) << (4 * b + r);
      }
    }
    if (__ballot(bits != 0)) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if ((bits >> (4 * b + r)) & 1) {
            const float G = acc[b][r];
            const float num = fmaf(G, qA[b] * cst[r].x, qB[b] * cst[r].y);
            float t = num * __builtin_amdgcn_rcpf(qQ[b] + cst[r].z);
            t = t > 0.0f ? t : 0.0f;
            float sc = fmaf(G, c1f, 0.35f) + t;
            sc = sc < 1.0f ? sc : 1.0f;
            sc = sc > 0.0f ? sc : 0.0f;  // +0 for -0 and negatives (k_sample_kth orders bit patterns)
            // sorted insert (descending), branch-free
#pragma unroll
            for (int u = 0; u < kTopT; ++u) {
              const float hi = fmaxf(top[b][u], sc);
              sc = fminf(top[b][u], sc);
              top[b][u] = hi;
            }
          }
        }
        k0[b] = ((qok >> b) & 1) ? 0.35f - top[b][kTopT - 1] : -__builtin_huge_valf();
      }
    }
    cf[0] = cf1[0];
    cf[1] = cf1[1];
    cf1[0] = cfn[0];
    cf1[1] = cfn[1];
    stv = st1;
    st1 = stn;
  }
  const int ns = 4 * a.nchunks;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    if (q >= a.Q) continue;
    float* o = a.top + ((int64_t)q * ns + 4 * chunk + g) * kTopT;
#pragma unroll
    for (int t = 0; t < kTopT; ++t) o[t] = top[b][t];
  }
}

// f32 sample pass, G-selected form (default): the step loop keeps, per lane (g, j) and query block b,
// only the step whose four rows 4g .. 4g + 3 hold the largest G (two v_max, one compare and six
// v_cndmask per block and step: the MFMA work sets the pace, as in k_scan0g), and scores the rows of
// that step exactly (f32 model) at the end; the stream's kTopT best of those scores go to the pool.  They
// are real scores of distinct (query, row) pairs, so the K-th best of the union is still a lower bound of
// the K-th best over the corpus (selecting by G instead of by score only makes it less tight).  Query
// constants and candidate statistics are read in the epilogue alone.  HI (default): the step loop
// contracts hi.hi only (the kept step is a heuristic choice) and the epilogue recomputes the kept rows'
// split G (split_g4) for the model score.
template <bool HI = true>
__global__ __launch_bounds__(64) void k_sample_topg(SampleArgs a) {
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.S) c_end = a.S;
  const int q0 = qb * kQW;
  half8 qh[4], ql[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const _Float16* zr = a.Zq16 + z16_frag(q < a.Q ? q : 0, g);
    qh[b] = *reinterpret_cast<const half8*>(zr);
    if constexpr (!HI) ql[b] = *reinterpret_cast<const half8*>(zr + kZ16Lo);
  }
  auto row_of = [&](int64_t i) -> int64_t { return sample_row_tiled(i, a.S, a.stride); };
  auto load_frag = [&](int64_t cs, half8* dst) {
    const _Float16* p = a.Zc16 + z16_frag(row_of(cs + j), g);
    HQ_GUARD(p, a.Zc16, z16_rows(a.N) * 64 - kZ16Lo - 8);
    dst[0] = *reinterpret_cast<const half8*>(p);
    if constexpr (!HI) dst[1] = *reinterpret_cast<const half8*>(p + kZ16Lo);
  };
  float bg[4];     // largest max-of-four G so far
  flt4 bacc[4];    // G of that step's four rows
  int bcs[4];      // that step (sample index of its first row), -1: none
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    bg[b] = -__builtin_huge_valf();
    bacc[b] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
    bcs[b] = -1;
  }
  half8 cf[2], cf1[2];
  load_frag(c_begin, cf);
  load_frag(c_begin + kCS, cf1);
  for (int64_t cs = c_begin; cs < c_end; cs += kCS) {
    half8 cfn[2];
    load_frag(cs + 2 * kCS, cfn);  // sample indices past S clamp to the last sample row
    flt4 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], qh[b], flt4{0, 0, 0, 0}, 0, 0, 0);
    if constexpr (!HI) {
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[0], ql[b], acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cf[1], qh[b], acc[b], 0, 0, 0);
    }
    if (cs + kCS > c_end) {  // the chunk's last, partial step: rows past c_end never win
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (cs + 4 * g + r >= c_end)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[b][r] = -__builtin_huge_valf();
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const float m = max4(acc[b]);
      const bool up = m > bg[b];
      bg[b] = up ? m : bg[b];
      bacc[b] = up ? acc[b] : bacc[b];
      bcs[b] = up ? (int)cs : bcs[b];
    }
    cf[0] = cf1[0];
    cf1[0] = cfn[0];
    if constexpr (!HI) {
      cf[1] = cf1[1];
      cf1[1] = cfn[1];
    }
  }
  // epilogue: exact f32 model scores of the selected rows, the stream's kTopT best to the pool.  Every
  // statistic is requested before any is used (one round trip): the four rows a lane scores per block are rows
  // 4g .. 4g + 3 of one sampled tile (steps start at tile boundaries), i.e. one SoA group of Sc32 — four
  // 16-byte loads; the query's four values likewise.  (The per-row form — flag load, test, then the row's
  // values — chained ~40 dependent loads through the epilogue: 82 waits, profiles/r06_pmc_sample_topg.txt.)
  const float c1f = (float)a.c1;
  const int ns = 4 * a.nchunks;
  flt4 qs4[4], sd4[4], mn4[4], ms4[4], fl4[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    const int qq = q < a.Q ? q : 0;
    const int64_t gq = (int64_t)(qq >> 2) * 16 + (qq & 3);  // SoA-per-4 statistics
    qs4[b] = flt4{a.Sq32[gq], a.Sq32[gq + 4], a.Sq32[gq + 8], a.Sq32[gq + 12]};
    const int64_t row0 = row_of((int64_t)(bcs[b] >= 0 ? bcs[b] : c_begin) + 4 * g);  // a multiple of 4
    const float* st = a.Sc32 + (row0 >> 2) * 16;
    HQ_GUARD(st, a.Sc32, pack0_rows(a.N) * 4 - 16);
    sd4[b] = *reinterpret_cast<const flt4*>(st);
    mn4[b] = *reinterpret_cast<const flt4*>(st + 4);
    ms4[b] = *reinterpret_cast<const flt4*>(st + 8);
    fl4[b] = *reinterpret_cast<const flt4*>(st + 12);
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int q = q0 + 16 * b + j;
    if (q >= a.Q) continue;
    const float qA = (float)(0.6 * a.inv_m) * qs4[b][0], qB = 0.6f * qs4[b][1], qQ = qs4[b][2];
    const bool qok = __float_as_int(qs4[b][3]) == 0;
    float top[kTopT];
#pragma unroll
    for (int t = 0; t < kTopT; ++t) top[t] = -1.0f;
    if (qok && bcs[b] >= 0) {
      flt4 Gs = bacc[b];
      if constexpr (HI) Gs = split_g4(a.Zq16, a.Zc16, q, row_of((int64_t)bcs[b] + 4 * g));  // 4 consecutive rows
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = (int64_t)bcs[b] + 4 * g + r;
        if (i >= c_end) continue;
        if (__float_as_int(fl4[b][r]) != 0) continue;  // flagged / pad row
        const float G = Gs[r];
        const float num = fmaf(G, qA * sd4[b][r], qB * mn4[b][r]);
        float t = num * __builtin_amdgcn_rcpf(qQ + ms4[b][r]);
        t = t > 0.0f ? t : 0.0f;
        float sc = fmaf(G, c1f, 0.35f) + t;
        sc = sc < 1.0f ? sc : 1.0f;
        sc = sc > 0.0f ? sc : 0.0f;  // +0 for -0 and negatives (k_sample_kth orders bit patterns)
#pragma unroll
        for (int u = 0; u < kTopT; ++u) {
          const float hi = fmaxf(top[u], sc);
          sc = fminf(top[u], sc);
          top[u] = hi;
        }
      }
    }
    float* o = a.top + ((int64_t)q * ns + 4 * chunk + g) * kTopT;
#pragma unroll
    for (int t = 0; t < kTopT; ++t) o[t] = top[t];
  }
}

// per-query starting threshold from the top-T sample pools (one wave per query): the K-th largest
// value v (bisection on the bit pattern of the non-negative f32 scores, pool held in registers as
// bits + 1, 0 = empty), th0 = v - margin, or -inf when fewer than K sample scores exist
constexpr int kKthReg = 32;  // pool entries per lane: 4 * 256 chunks * kTopT / 64

// Also clears the scan's per-query published threshold and pool count (gtau, pool_n; top-T mode has no
// histogram, so no memset runs before the scan).
template <int R>
__global__ __launch_bounds__(64) void k_sample_kth(const float* __restrict__ top, int ns, int Q, int K, double margin,
                                                   double* __restrict__ th0, unsigned long long* __restrict__ gtau,
                                                   int* __restrict__ pool_n, const float* __restrict__ Sq32, double thr0,
                                                   double inv_m, QConst* __restrict__ qc) {
  const int lane = threadIdx.x;
  const int P = ns * kTopT;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    if (lane == 0) {
      if (gtau) gtau[q] = 0ull;
      pool_n[q] = 0;
    }
    const float* p = top + (int64_t)q * P;
    // the query's statistics for its constants, requested with the pool (one round trip)
    float st[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (qc && lane == 0) {
      const int64_t gq = (int64_t)(q >> 2) * 16 + (q & 3);
#pragma unroll
      for (int e = 0; e < 4; ++e) st[e] = Sq32[gq + 4 * e];
    }
    uint32_t u[R];
#pragma unroll
    for (int e = 0; e < R; ++e) {
      const int x = lane + 64 * e;
      const float v = x < P ? p[x] : -1.0f;
      u[e] = v >= 0.0f ? __float_as_uint(v) + 1u : 0u;
    }
    auto count_ge = [&](uint32_t t) {  // entries with u >= t (t >= 1): DPP sum, no LDS round trips
      int c = 0;
#pragma unroll
      for (int e = 0; e < R; ++e) c += u[e] >= t ? 1 : 0;
      return wsum64i(c);
    };
    double t = -__builtin_huge_val();
    if (count_ge(1u) >= K) {
      uint32_t lo = 1u, hi = 0x3F800002u;  // count_ge(lo) >= K, count_ge(hi) < K (scores <= 1)
      while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (count_ge(mid) >= K) lo = mid; else hi = mid;
      }
      t = (double)__uint_as_float(lo - 1u) - margin;
    }
    if (lane == 0) {
      th0[q] = t;
      if (qc) qc[q] = qconst_vals(st[0], st[1], st[2], __float_as_int(st[3]), t > thr0 ? t : thr0, inv_m);
    }
  }
}

// the pool held in registers: R = 8 / 16 / 32 entries per lane (ns * kTopT <= 64 R; the geometry caps it
// at 64 kKthReg), so a smaller pool makes every bisection step cheaper
static void launch_kth(int mg, hipStream_t s, const float* top, int ns, int Q, int K, double margin, double* th0,
                       unsigned long long* gtau, int* pool_n, const float* Sq32, double thr0, double inv_m,
                       QConst* qc) {
  const int P = ns * kTopT;
  if (P <= 64 * 8)
    hipLaunchKernelGGL(k_sample_kth<8>, dim3(mg), dim3(64), 0, s, top, ns, Q, K, margin, th0, gtau, pool_n, Sq32, thr0,
                       inv_m, qc);
  else if (P <= 64 * 16)
    hipLaunchKernelGGL(k_sample_kth<16>, dim3(mg), dim3(64), 0, s, top, ns, Q, K, margin, th0, gtau, pool_n, Sq32,
                       thr0, inv_m, qc);
  else
    hipLaunchKernelGGL(k_sample_kth<kKthReg>, dim3(mg), dim3(64), 0, s, top, ns, Q, K, margin, th0, gtau, pool_n, Sq32,
                       thr0, inv_m, qc);
}

#ifdef HQ_DIAG
// per-query starting threshold from the sample histogram (-inf when the sample has < K scores)
__global__ void k_hist_tau(const unsigned int* __restrict__ hist, int Q, int K, double margin,
                           double* __restrict__ th0) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  unsigned int cum = 0;
  double t = -__builtin_huge_val();
  for (int e = kBins - 1; e >= 0; --e) {
    cum += hist[(int64_t)q * kBins + e];
    if (cum >= (unsigned int)K) {
      t = (double)e / (double)kBins - margin;  // margin > the score error of the sample pass
      break;
    }
  }
  th0[q] = t;
}
#endif  // HQ_DIAG

// merge nchunks sorted lists per query (one wave per query)
__global__ __launch_bounds__(64) void k_merge(const double* __restrict__ ws_score, const int64_t* __restrict__ ws_id,
                                              const double* __restrict__ ws_best, const int64_t* __restrict__ ws_best_id,
                                              int nchunks, int Q, int K, double* __restrict__ out_score,
                                              int64_t* __restrict__ out_id, double* __restrict__ out_best,
                                              int64_t* __restrict__ out_best_id) {
  const int lane = threadIdx.x;
  constexpr int kPerLane = 8;  // nchunks <= 512
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    int head[kPerLane];
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) head[i] = 0;
    for (int j = 0; j < K; ++j) {
      // this lane's best head
      double s = -__builtin_huge_val();
      int64_t id = -1;
      int which = -1;
#pragma unroll
      for (int i = 0; i < kPerLane; ++i) {
        const int c = lane + 64 * i;
        if (c < nchunks && head[i] < K) {
          const int64_t o = ((int64_t)c * Q + q) * K + head[i];
          const int64_t id2 = ws_id[o];
          const double s2 = ws_score[o];
          if (id2 >= 0 && (id < 0 || better(s2, id2, s, id))) { s = s2; id = id2; which = i; }
        }
      }
      double bs = s;
      int64_t bid = id;
      for (int o = 1; o < 64; o <<= 1) {
        const double s2 = __shfl_xor(bs, o, 64);
        const int64_t id2 = __shfl_xor(bid, o, 64);
        if (id2 >= 0 && (bid < 0 || better(s2, id2, bs, bid))) { bs = s2; bid = id2; }
      }
      if (bid >= 0 && id == bid && which >= 0) {
#pragma unroll
        for (int i = 0; i < kPerLane; ++i)
          if (i == which) head[i]++;
      }
      if (lane == 0) {
        out_score[(int64_t)q * K + j] = bid >= 0 ? bs : -__builtin_huge_val();
        out_id[(int64_t)q * K + j] = bid;
      }
    }
    if (out_best) {
      double s = -__builtin_huge_val();
      int64_t id = -1;
      for (int c = lane; c < nchunks; c += 64) {
        const double s2 = ws_best[(int64_t)c * Q + q];
        const int64_t id2 = ws_best_id[(int64_t)c * Q + q];
        if (id2 >= 0 && (id < 0 || better(s2, id2, s, id))) { s = s2; id = id2; }
      }
      for (int o = 1; o < 64; o <<= 1) {
        const double s2 = __shfl_xor(s, o, 64);
        const int64_t id2 = __shfl_xor(id, o, 64);
        if (id2 >= 0 && (id < 0 || better(s2, id2, s, id))) { s = s2; id = id2; }
      }
      if (lane == 0) { out_best[q] = s; out_best_id[q] = id; }
    }
  }
}

// progressive search final stage (search_engine.py:284-298 fallback, :340-388 re-rank), R-way,
// one wave per query.  lists are sorted by (level-0 score desc, id asc); det rows are
// [overall, level sims...].  Survivors = global top-M of the R lists (merged on (score, id), as the
// reference's stable sort over the pool order); if none, the first arg-max of the level-0 score;
// then a stable sort by overall score (ties keep the level-0 order) and the first K.
__device__ __forceinline__ bool wave_better(double s, int64_t id, double s2, int64_t id2) {
  return id >= 0 && (id2 < 0 || s > s2 || (s == s2 && id < id2));
}

// survivors of query q (one wave, no barrier inside: callers synchronise before reading sel): the global
// top-M of the R lists merged on (score desc, id asc) into sel[] as (list r << 16) | slot; if none passed,
// the first arg-max of the level-0 score (sel[0] = r << 16, *fb_id = its id).  Returns the count.
__device__ int final_survivors(int R, int Q, int M, int q, const double* __restrict__ s0,
                               const int64_t* __restrict__ ids, const double* __restrict__ best,
                               const int64_t* __restrict__ best_id, int* sel, int64_t* fb_id, bool k32) {
  const int lane = threadIdx.x & 63;
  // ---- R-way merge: lane r < R follows list r's head ----
  int h = 0;
  double hs = -__builtin_huge_val();
  int64_t hid = -1;
  auto load_head = [&]() {
    hs = -__builtin_huge_val();
    hid = -1;
    if (lane < R && h < M) {
      const int64_t o = ((int64_t)lane * Q + q) * M + h;
      hid = ids[o];
      if (hid >= 0) hs = key_of(s0[o], k32);
    }
  };
  load_head();
  int n = 0;
  if (R == 1) {
    // one list: it is already the (score desc, id asc) order; its valid entries come first
    for (int i = lane; i < M; i += 64) {
      const bool v = ids[(int64_t)q * M + i] >= 0;
      const unsigned long long m = __ballot(v);
      n += __popcll(m);
      if (v) sel[i] = i;
    }
    n = __builtin_amdgcn_readfirstlane(n);
  }
  for (; R > 1 && n < M; ++n) {
    double bs = hs;
    int64_t bid = hid;
    int bl = lane;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bid, o, 64);
      const int l2 = __shfl_xor(bl, o, 64);
      if (wave_better(s2, i2, bs, bid)) { bs = s2; bid = i2; bl = l2; }
    }
    if (bid < 0) break;
    const int hb = __shfl(h, bl, 64);
    if (lane == 0) sel[n] = (bl << 16) | hb;
    if (lane == bl) {
      h = hb + 1;
      load_head();
    }
  }
  *fb_id = -1;
  if (n == 0) {
    // none passed the threshold: keep the first arg-max of the level-0 score (:295-298)
    double bs = -__builtin_huge_val();
    int64_t bid = -1;
    int bl = lane;
    if (lane < R) {
      bid = best_id[(int64_t)lane * Q + q];
      if (bid >= 0) bs = key_of(best[(int64_t)lane * Q + q], k32);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bid, o, 64);
      const int l2 = __shfl_xor(bl, o, 64);
      if (wave_better(s2, i2, bs, bid)) { bs = s2; bid = i2; bl = l2; }
    }
    if (bid >= 0) {
      n = 1;
      *fb_id = bid;
      if (lane == 0) sel[0] = bl << 16;
    }
  }
  return n;
}

__global__ __launch_bounds__(64) void k_progressive_final(int R, int Q, int M, int W, const double* __restrict__ s0,
                                                          const int64_t* __restrict__ ids,
                                                          const double* __restrict__ det,
                                                          const double* __restrict__ best,
                                                          const int64_t* __restrict__ best_id,
                                                          const double* __restrict__ best_det, int K,
                                                          int64_t* __restrict__ out_id, double* __restrict__ out_det,
                                                          int* __restrict__ out_count, int flags) {
  __shared__ int sel[kMaxFinal];  // survivor i -> (list r << 16) | slot
  const int lane = threadIdx.x;
  const bool k32 = (flags & 1) != 0;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    int64_t fb_id;
    const int n = final_survivors(R, Q, M, q, s0, ids, best, best_id, sel, &fb_id, k32);
    __syncthreads();
    const double* rowbase = fb_id >= 0 ? best_det : det;
    // ---- stable sort of the survivors by overall score ----
    const int outn = n < K ? n : K;
    // row of survivor i in rowbase: list rows (r Q + q) M + slot, or the fallback's best row r Q + q
    auto row_of = [&](int v) -> int64_t {
      const int64_t rq = (int64_t)(v >> 16) * Q + q;
      return fb_id >= 0 ? rq : rq * M + (v & 0xFFFF);
    };
    // stable rank of survivor i: ranks from register copies of the overall scores (n <= 64 here:
    // M <= 64 on the fused path; larger n re-reads the rows)
    double ovl = -__builtin_huge_val();
    if (lane < n) ovl = key_of(rowbase[row_of(sel[lane]) * W], k32);
    for (int i = lane; i < n; i += 64) {
      const int64_t oi = row_of(sel[i]);
      const double ovi = key_of(rowbase[oi * W], k32);
      int rank = 0;
      if (n <= 64) {
        for (int jj = 0; jj < n; ++jj) {
          const double ovj = rl_f64(ovl, jj);
          rank += (ovj > ovi || (ovj == ovi && jj < i)) ? 1 : 0;
        }
      } else {
        for (int jj = 0; jj < n; ++jj) {
          const double ovj = key_of(rowbase[row_of(sel[jj]) * W], k32);
          rank += (ovj > ovi || (ovj == ovi && jj < i)) ? 1 : 0;
        }
      }
      if (rank < K) {
        out_id[(int64_t)q * K + rank] = fb_id >= 0 ? fb_id : ids[oi];
        for (int w = 0; w < W; ++w) out_det[((int64_t)q * K + rank) * W + w] = rowbase[oi * W + w];
      }
    }
    for (int i = outn + lane; i < K; i += 64) {
      out_id[(int64_t)q * K + i] = -1;
      for (int w = 0; w < W; ++w) out_det[((int64_t)q * K + i) * W + w] = 0.0;
    }
    if (lane == 0) out_count[q] = outn;
    __syncthreads();
  }
}


// top-k of a dense score matrix per query (one wave per query): (score desc, id asc) with the
// threshold test, plus the first arg-max over all candidates.  Used when k exceeds the fused
// scan's LDS lists (e.g. the reference engine's default max_candidates_per_level = 100).
// Top-k (score desc, id asc) of one candidate row among entries passing the threshold test, plus the
// first arg-max over all entries; one wave.  Candidate c has id rid[c] (rid != NULL; -1 = empty) or c;
// ids are written with id_base added.  k passes, each after the previous pick in the total order.
__device__ void select_row(const double* __restrict__ row, const int64_t* __restrict__ rid, int64_t n, int k,
                           double thr, int thr_mode, int64_t id_base, double* __restrict__ out_s,
                           int64_t* __restrict__ out_id, double* __restrict__ best, int64_t* __restrict__ best_id) {
  const int lane = threadIdx.x & 63;
  double ps = __builtin_huge_val();
  int64_t pid = -1;
  for (int j = 0; j < k; ++j) {
    double bs = 0.0;
    int64_t bi = -1;
    for (int64_t c = lane; c < n; c += 64) {
      const int64_t id = rid ? rid[c] : c;
      if (id < 0) continue;
      const double s = row[c];
      const bool ok = thr_mode == 0 || (thr_mode == 1 ? s >= thr : s > thr);
      if (!ok) continue;
      if (pid >= 0 && !better(ps, pid, s, id)) continue;  // must come after the previous pick
      if (bi < 0 || better(s, id, bs, bi)) { bs = s; bi = id; }
    }
    for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bi, o, 64);
      if (i2 >= 0 && (bi < 0 || better(s2, i2, bs, bi))) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      out_s[j] = bi >= 0 ? bs : -__builtin_huge_val();
      out_id[j] = bi >= 0 ? bi + id_base : -1;
    }
    if (bi < 0) {
      for (int jj = j + 1 + lane; jj < k; jj += 64) {
        out_s[jj] = -__builtin_huge_val();
        out_id[jj] = -1;
      }
      break;
    }
    ps = bs;
    pid = bi;
  }
  if (best) {
    double bs = 0.0;
    int64_t bi = -1;
    for (int64_t c = lane; c < n; c += 64) {
      const int64_t id = rid ? rid[c] : c;
      if (id < 0) continue;
      if (bi < 0 || better(row[c], id, bs, bi)) { bs = row[c]; bi = id; }
    }
    for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bi, o, 64);
      if (i2 >= 0 && (bi < 0 || better(s2, i2, bs, bi))) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      *best = bi >= 0 ? bs : -__builtin_huge_val();
      *best_id = bi >= 0 ? bi + id_base : -1;
    }
  }
}

__global__ __launch_bounds__(64) void k_select(const double* __restrict__ sc, int Q, int64_t N, int k, double thr,
                                               int thr_mode, int64_t id_base, double* __restrict__ out_s,
                                               int64_t* __restrict__ out_id, double* __restrict__ best,
                                               int64_t* __restrict__ best_id) {
  for (int q = blockIdx.x; q < Q; q += gridDim.x)
    select_row(sc + (int64_t)q * N, nullptr, N, k, thr, thr_mode, id_base, out_s + (int64_t)q * k,
               out_id + (int64_t)q * k, best ? best + q : nullptr, best ? best_id + q : nullptr);
}

// Two-stage select for long rows: stage 1, one wave per (query, part of plen entries): the part's
// top-k and arg-max with row-local ids into the workspace; stage 2 (k_select_merge): the same
// selection over each query's P x k candidates (ids carried) and P arg-maxes.  The total order is the
// same, so the result equals the one-stage select.
__global__ __launch_bounds__(64) void k_select_part(const double* __restrict__ sc, int Q, int64_t N, int P,
                                                    int64_t plen, int k, double thr, int thr_mode,
                                                    double* __restrict__ ws_s, int64_t* __restrict__ ws_id,
                                                    double* __restrict__ ws_b, int64_t* __restrict__ ws_bid) {
  for (int64_t t = blockIdx.x; t < (int64_t)Q * P; t += gridDim.x) {
    const int64_t q = t / P, p = t % P;
    const int64_t c0 = p * plen;
    const int64_t n = c0 >= N ? 0 : (N - c0 < plen ? N - c0 : plen);
    select_row(sc + q * N + c0, nullptr, n, k, thr, thr_mode, c0, ws_s + t * k, ws_id + t * k, ws_b + t,
               ws_bid + t);
  }
}

__global__ __launch_bounds__(64) void k_select_merge(int Q, int P, int k, double thr, int thr_mode, int64_t id_base,
                                                     const double* __restrict__ ws_s,
                                                     const int64_t* __restrict__ ws_id,
                                                     const double* __restrict__ ws_b,
                                                     const int64_t* __restrict__ ws_bid, double* __restrict__ out_s,
                                                     int64_t* __restrict__ out_id, double* __restrict__ best,
                                                     int64_t* __restrict__ best_id) {
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    const int64_t o = (int64_t)q * P * k;
    select_row(ws_s + o, ws_id + o, (int64_t)P * k, k, thr, thr_mode, id_base, out_s + (int64_t)q * k,
               out_id + (int64_t)q * k, nullptr, nullptr);
    if (best) {
      // arg-max of the part arg-maxes: thr_mode 0 top-1 over (score, id) = the first arg-max
      select_row(ws_b + (int64_t)q * P, ws_bid + (int64_t)q * P, P, 1, 0.0, 0, id_base, best + q, best_id + q,
                 nullptr, nullptr);
    }
  }
}

// Register-resident multi-stage select for few queries (the dense redo of a handful of queries: the
// two-stage form above then runs only N / 8192 waves per query, each making k passes over its part in
// memory — 1.1 ms for one 1M-entry row).  Stage 1: one wave per (query, part of kRegSel entries) holds
// its entries in registers (kSelR per lane) and makes the k passes there; merge stages take fan-in F
// parts' candidates the same way until one part remains.  Same total order (score desc, row asc), same
// threshold test and first arg-max as select_row, so the result is identical.
constexpr int kSelR = 16;
constexpr int kRegSel = 64 * kSelR;

__device__ __forceinline__ void wave_best(double& bs, int64_t& bi) {
  for (int o = 1; o < 64; o <<= 1) {
    const double s2 = __shfl_xor(bs, o, 64);
    const int64_t i2 = __shfl_xor(bi, o, 64);
    if (i2 >= 0 && (bi < 0 || better(s2, i2, bs, bi))) { bs = s2; bi = i2; }
  }
}

// k passes over the wave's register entries (id < 0: empty): (score, id + id_add), padded with -inf / -1
__device__ __forceinline__ void reg_topk(const double (&s)[kSelR], const int64_t (&id)[kSelR], int k, int64_t id_add,
                                         double* __restrict__ out_s, int64_t* __restrict__ out_id) {
  const int lane = threadIdx.x & 63;
  double ps = __builtin_huge_val();
  int64_t pid = -1;
  for (int j = 0; j < k; ++j) {
    double bs = 0.0;
    int64_t bi = -1;
#pragma unroll
    for (int r = 0; r < kSelR; ++r) {
      const bool after = pid < 0 || better(ps, pid, s[r], id[r]);  // must come after the previous pick
      if (id[r] >= 0 && after && (bi < 0 || better(s[r], id[r], bs, bi))) { bs = s[r]; bi = id[r]; }
    }
    wave_best(bs, bi);
    if (lane == 0) {
      out_s[j] = bi >= 0 ? bs : -__builtin_huge_val();
      out_id[j] = bi >= 0 ? bi + id_add : -1;
    }
    if (bi < 0) {
      for (int jj = j + 1 + lane; jj < k; jj += 64) {
        out_s[jj] = -__builtin_huge_val();
        out_id[jj] = -1;
      }
      break;
    }
    ps = bs;
    pid = bi;
  }
}

// stage 1: parts of a dense [Q, N] row; ids = row index (+ id_add when this is the last stage)
__global__ __launch_bounds__(64) void k_select_reg1(const double* __restrict__ sc, int Q, int64_t N, int P, int k,
                                                    double thr, int thr_mode, int64_t id_add,
                                                    double* __restrict__ o_s, int64_t* __restrict__ o_id,
                                                    double* __restrict__ o_b, int64_t* __restrict__ o_bid) {
  const int lane = threadIdx.x;
  for (int64_t t = blockIdx.x; t < (int64_t)Q * P; t += gridDim.x) {
    const int64_t q = t / P, c0 = (t % P) * kRegSel;
    double s[kSelR];
    int64_t id[kSelR];
    double bs = 0.0;
    int64_t bi = -1;  // first arg-max over every entry (no threshold)
#pragma unroll
    for (int r = 0; r < kSelR; ++r) {
      const int64_t c = c0 + lane + 64 * r;
      const bool valid = c < N;
      const double v = valid ? sc[q * N + c] : 0.0;
      if (valid && (bi < 0 || better(v, c, bs, bi))) { bs = v; bi = c; }
      const bool pass = thr_mode == 0 || (thr_mode == 1 ? v >= thr : v > thr);
      s[r] = v;
      id[r] = valid && pass ? c : -1;
    }
    wave_best(bs, bi);
    if (lane == 0 && o_b) {
      o_b[t] = bi >= 0 ? bs : -__builtin_huge_val();
      o_bid[t] = bi >= 0 ? bi + id_add : -1;
    }
    reg_topk(s, id, k, id_add, o_s + t * k, o_id + t * k);
  }
}

// merge stage: group g of query q = parts [g F, g F + F) of the previous stage (P parts) -> one part
__global__ __launch_bounds__(64) void k_select_regm(int Q, int P, int F, int P2, int k, int64_t id_add,
                                                    const double* __restrict__ i_s, const int64_t* __restrict__ i_id,
                                                    const double* __restrict__ i_b, const int64_t* __restrict__ i_bid,
                                                    double* __restrict__ o_s, int64_t* __restrict__ o_id,
                                                    double* __restrict__ o_b, int64_t* __restrict__ o_bid) {
  const int lane = threadIdx.x;
  for (int64_t t = blockIdx.x; t < (int64_t)Q * P2; t += gridDim.x) {
    const int64_t q = t / P2, p0 = (t % P2) * F;
    const int np = (int)(P - p0 < F ? P - p0 : F);
    const int64_t base = (q * P + p0) * k;
    double s[kSelR];
    int64_t id[kSelR];
#pragma unroll
    for (int r = 0; r < kSelR; ++r) {
      const int e = lane + 64 * r;
      const bool valid = e < np * k;
      s[r] = valid ? i_s[base + e] : 0.0;
      id[r] = valid ? i_id[base + e] : -1;  // threshold already applied in stage 1
    }
    reg_topk(s, id, k, id_add, o_s + t * k, o_id + t * k);
    if (o_b) {
      double bs = 0.0;
      int64_t bi = -1;
      if (lane < np) {
        const int64_t i = i_bid[q * P + p0 + lane];
        if (i >= 0) { bs = i_b[q * P + p0 + lane]; bi = i; }
      }
      wave_best(bs, bi);
      if (lane == 0) {
        o_b[t] = bi >= 0 ? bs : -__builtin_huge_val();
        o_bid[t] = bi >= 0 ? bi + id_add : -1;
      }
    }
  }
}

// compare_indices_at_level on raw equal-length segments (mixed-length candidate pools): the query
// segment q[0..m) against each row of C (N x m), statistics computed in place in NumPy order and in each
// side's dtype (q_f32 / c_f32: float32 values).
__global__ __launch_bounds__(256) void k_pair_raw(const double* __restrict__ q, const double* __restrict__ C, int64_t N,
                                                  int m, int q_f32, int c_f32, double* __restrict__ out) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    int t32;
    out[c] = exact_level_sides(make_side(q, nullptr, nullptr, m, q_f32 != 0),
                               make_side(C + c * m, nullptr, nullptr, m, c_f32 != 0), m, &t32);
  }
}

// Exact re-rank of an approximate (MFMA) candidate list, one wave per query.  cand lists [Q, kp] are
// sorted by approximate score (id -1 = empty slot).  Output: the exact top-k (score desc, id asc)
// among listed candidates passing the exact threshold test, their count, and resolved = 1 when no
// unlisted candidate can belong to the exact top-k given |approx - exact| <= eps:
//   list not full (every candidate with approx >= thr - eps is listed), or
//   last listed approx + eps < k-th exact score (enough passed), or < / <= thr (too few passed).
template <bool SM = false>
__global__ __launch_bounds__(64) void k_refine(VecSet Qs, int Q, VecSet Cs, int64_t N, SegInfo si, int mode,
                                               const double* __restrict__ cs, const int64_t* __restrict__ cid, int kp,
                                               int k, double thr, int thr_mode, double eps, int64_t id_base,
                                               double* __restrict__ os, int64_t* __restrict__ oid,
                                               int* __restrict__ ocnt, int* __restrict__ ores, int count_empty,
                                               int* __restrict__ oredo, int* __restrict__ onext) {
  __shared__ double es[kMaxTopK];
  if (onext && blockIdx.x == 0 && threadIdx.x == 0) *onext = 0;  // the next batch's redo counter
  __shared__ int64_t ei[kMaxTopK];
  const int lane = threadIdx.x;
  const bool k32 = (thr_mode & kThrKey32) != 0;
  thr_mode &= kThrKey32 - 1;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    const int64_t base = (int64_t)q * kp;
    if (lane < kp) {
      double e = -__builtin_huge_val();
      int64_t id = cid[base + lane];
      const int64_t c = id - id_base;
      if (id >= 0 && c >= 0 && c < N) {
        int typed = 0;
        e = exact_pair<SM>(Qs, q, Cs, c, si, mode == 0 ? 0 : -1, nullptr, &typed);
        const bool pass = mode == 0 ? typed_pass(e, typed, thr, thr_mode)
                                    : (thr_mode == 0 || (thr_mode == 1 ? e >= thr : e > thr));
        if (!pass) id = -1;
      } else {
        id = -1;
      }
      es[lane] = e;
      ei[lane] = id;
    }
    __syncthreads();
    // rank of each valid entry by (score desc, id asc) among the valid ones (kp <= 64: one lane each)
    const double e = lane < kp ? es[lane] : -__builtin_huge_val();
    const double ek = key_of(e, k32);
    const int64_t id = lane < kp ? ei[lane] : -1;
    const bool valid = id >= 0;
    const int n = __popcll(__ballot(valid));
    int rank = 0;
    for (int o = 0; o < kp; ++o) {
      const double so = rl_f64(ek, o);
      const long long io = __double_as_longlong(rl_f64(__longlong_as_double((long long)id), o));
      rank += (io >= 0 && (so > ek || (so == ek && io < id))) ? 1 : 0;
    }
    const int cnt = n < k ? n : k;
    if (valid && rank < k) {
      os[(int64_t)q * k + rank] = e;
      oid[(int64_t)q * k + rank] = id;
    }
    for (int j = cnt + lane; j < k; j += 64) {
      os[(int64_t)q * k + j] = -__builtin_huge_val();
      oid[(int64_t)q * k + j] = -1;
    }
    // k-th exact score (the entry of rank k - 1)
    const unsigned long long mk = __ballot(valid && rank == k - 1);
    const double kth = mk ? rl_f64(e, __builtin_ctzll(mk)) : -__builtin_huge_val();
    if (lane == 0) {
      ocnt[q] = cnt;
      const bool full = cid[base + kp - 1] >= 0;
      // an empty last slot with score +inf: the scan's list may be incomplete (k_pool_select)
      const bool trunc = !full && cs[base + kp - 1] == __builtin_huge_val();
      int res = trunc ? 0 : 1;
      if (full) {
        const double bound = cs[base + kp - 1] + eps;
        if (n >= k) res = k32 ? (float)bound < (float)kth : bound < kth;
        else if (thr_mode == 0) res = 0;
        else res = thr_mode == 1 ? (bound < thr_low(thr)) : (bound <= thr_low(thr));
      }
      ores[q] = res;
      if (oredo && (res == 0 || (count_empty && cnt == 0))) atomicAdd(oredo, 1);
    }
    __syncthreads();
  }
}

// LDS-staged exact re-rank (default when the rows fit): one wave per query copies the query's and the
// kp listed candidates' rows (raw [L], Z [Lp], S [nseg x 4] = RW doubles each) into LDS with all loads
// in flight at once (8 per lane per round), then scores from LDS, so the random corpus rows cost one
// memory round trip instead of one per dependent load.  Same contract and arithmetic as k_refine (the
// same exact_pair code on other addresses).  odet != NULL: also the exact [overall, level 0..] record of
// every output entry (hq_rescore's values for the output ids, zeros for empty slots), from the rows
// already staged - the progressive search then needs no separate re-score launch.
// staged doubles: the query row (raw [L], Z [Lp], S [nseg x 4]) and kp candidate rows of raw + S (a
// candidate's normalised values are recomputed as (x - mean) / std from its statistics: the same f64
// operations k_seg_prepare stored in Z, so bit-identical, and 45% fewer bytes gathered)
__host__ __device__ inline int refine_rw(const SegInfo& si) { return si.L + 4 * si.nseg; }
__host__ __device__ inline int refine_qw(const SegInfo& si) { return si.L + si.Lp + 4 * si.nseg; }
// every level segment <= 128 values: the exact scorers' NumPy sums are single pairwise leaves (SM kernels)
inline bool seg_small(const SegInfo& si) {
  for (int s = 0; s < si.nseg; ++s)
    if (si.len[s] > 128) return false;
  return true;
}

// nbytes (multiple of 16) from g to LDS byte address d (16-B aligned) by LDS-DMA, 1 KiB per instruction
__device__ __forceinline__ void dma_seg(const double* g, uint32_t d, int nbytes, int lane) {
  for (int off = 0; off < nbytes; off += 1024) {
    if (off + 16 * lane < nbytes) {
      uint32_t keep;
      const char* src = reinterpret_cast<const char*>(g) + off + 16 * lane;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(d + (uint32_t)off)) : "memory");
    }
  }
}

// the reference's typed weighted sum of the level scores (search_engine.py:191-230; see exact_pair_rows)
__device__ __forceinline__ double overall_from_levels(const double* lv, const int* t32, int nseg) {
  double tws = 0.0, tw = 0.0;
  bool acc32 = false;
  for (int s = 0; s < nseg; ++s) {
    const double w = 1.0 / (double)(s + 1);
    const double term = t32[s] ? (double)((float)lv[s] * (float)w) : lv[s] * w;
    if (!acc32 && !t32[s]) {
      tws = tws + term;
    } else {
      tws = (double)((float)tws + (float)term);
      acc32 = true;
    }
    tw = tw + w;
  }
  double ov;
  if (acc32) {
    const float o = (float)tws / (float)tw;
    ov = o < 1.0f ? (double)o : 1.0;
  } else {
    ov = tw > 0.0 ? tws / tw : 0.0;
    ov = ov < 1.0 ? ov : 1.0;
  }
  return ov > 0.0 ? ov : 0.0;
}

// One 256-thread workgroup per query: the four waves stage the rows by LDS-DMA (wave w: rows w, w + 4,
// ...), then every (candidate, level) score is one task over the 256 threads in level-major order (the
// long level-0 tasks all in the first round), wave 0 adds each candidate's levels in the reference's
// order and typing, ranks and writes.  Needed tasks: level 0 only for mode 0 without odet.
#define HQ_REFINE_ARGS                                                                                        \
  VecSet Qs, int Q, VecSet Cs, int64_t N, SegInfo si, int mode, const double *__restrict__ cs,                  \
      const int64_t *__restrict__ cid, int kp, int k, double thr, int thr_mode, double eps, int64_t id_base,     \
      double *__restrict__ os, int64_t *__restrict__ oid, int *__restrict__ ocnt, int *__restrict__ ores,        \
      int count_empty, int *__restrict__ oredo, double *__restrict__ odet, int expt,     \
      int *__restrict__ onext
#define HQ_REFINE_PASS Qs, Q, Cs, N, si, mode, cs, cid, kp, k, thr, thr_mode, eps, id_base, os, oid, ocnt, ores, count_empty, oredo, odet, expt, onext
template <bool SM>
__device__ __forceinline__ void refine_lds_body(HQ_REFINE_ARGS) {
  if (onext && blockIdx.x == 0 && threadIdx.x == 0) *onext = 0;  // the next batch's redo counter
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ int64_t srow[kMaxTopK + 1];  // source row per staged row (-1: empty)
  __shared__ int t32s[kMaxTopK * kMaxSeg];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int RW = refine_rw(si), QW = refine_qw(si), W = 1 + si.nseg, nr = kp + 1;
  double* rq = sm;                            // query row: raw, Z, S
  double* rows = sm + QW;                     // kp x RW candidate rows: raw, S
  double* lvs = rows + (int64_t)kp * RW;      // kp x W: overall, levels
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)sm;
  const int nlev = (mode == 0 && !odet) ? 1 : si.nseg;
  const bool k32 = (thr_mode & kThrKey32) != 0;
  thr_mode &= kThrKey32 - 1;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    const int64_t base = (int64_t)q * kp;
    if (tid < nr) {
      int64_t r = q;
      if (tid > 0) {
        const int64_t id = cid[base + tid - 1];
        const int64_t c = id - id_base;
        r = (id >= 0 && c >= 0 && c < N) ? c : -1;
      }
      srow[tid] = r;
    }
    __syncthreads();
    // stage by LDS-DMA (global_load_lds_dwordx4: lane l writes 16 B at m0 + 16 l), all pieces in flight
    for (int r = wave; r < nr && expt != 1; r += 4) {  // expt: diagnostics (1 no staging, 2 no scoring)
      const int64_t i = srow[r];
      if (i < 0) continue;
      if (r == 0) {
        dma_seg(Qs.raw + i * si.L, lbase, 8 * si.L, lane);
        dma_seg(Qs.Z + i * si.Lp, lbase + 8u * si.L, 8 * si.Lp, lane);
        dma_seg(Qs.S + i * si.nseg * 4, lbase + 8u * (si.L + si.Lp), 32 * si.nseg, lane);
      } else {
        const uint32_t d0 = lbase + 8u * (uint32_t)(QW + (r - 1) * RW);
        dma_seg(Cs.raw + i * si.L, d0, 8 * si.L, lane);
        dma_seg(Cs.S + i * si.nseg * 4, d0 + 8u * si.L, 32 * si.nseg, lane);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // level scores: task t = s * kp + p
    for (int t = tid; t < nlev * kp && expt != 2; t += 256) {
      const int sg = t / kp, p = t - sg * kp;
      double v = 0.0;
      int f32 = 0;
      if (srow[p + 1] >= 0) {
        const double* rc = rows + (int64_t)p * RW;
        v = exact_level<SM>(rq + si.src[sg], rq + si.L + si.poff[sg], rq + si.L + si.Lp + 4 * sg, rc + si.src[sg],
                            nullptr, rc + si.L + 4 * sg, si.len[sg], &f32);
      }
      lvs[(int64_t)p * W + 1 + sg] = v;
      t32s[p * kMaxSeg + sg] = f32;
    }
    __syncthreads();
    if (wave == 0) {
      double e = -__builtin_huge_val();
      int64_t id = -1;
      if (lane < kp) {
        id = cid[base + lane];
        if (srow[lane + 1] >= 0) {
          double* lv = lvs + (int64_t)lane * W;
          const double ov = nlev == si.nseg ? overall_from_levels(lv + 1, t32s + lane * kMaxSeg, si.nseg) : 0.0;
          lv[0] = ov;
          e = mode == 0 ? lv[1] : ov;
          const bool pass = mode == 0 ? typed_pass(e, t32s[lane * kMaxSeg], thr, thr_mode)
                                      : (thr_mode == 0 || (thr_mode == 1 ? e >= thr : e > thr));
          if (!pass) id = -1;
        } else {
          id = -1;
        }
      }
      const bool valid = id >= 0;
      const int n = __popcll(__ballot(valid));
      const double ek = key_of(e, k32);
      int rank = 0;
      for (int o = 0; o < kp; ++o) {
        const double so = rl_f64(ek, o);
        const long long io = __double_as_longlong(rl_f64(__longlong_as_double((long long)id), o));
        rank += (io >= 0 && (so > ek || (so == ek && io < id))) ? 1 : 0;
      }
      const int cnt = n < k ? n : k;
      if (valid && rank < k) {
        os[(int64_t)q * k + rank] = e;
        oid[(int64_t)q * k + rank] = id;
        if (odet)
          for (int w = 0; w < W; ++w) odet[((int64_t)q * k + rank) * W + w] = lvs[(int64_t)lane * W + w];
      }
      for (int j = cnt + lane; j < k; j += 64) {
        os[(int64_t)q * k + j] = -__builtin_huge_val();
        oid[(int64_t)q * k + j] = -1;
        if (odet)
          for (int w = 0; w < W; ++w) odet[((int64_t)q * k + j) * W + w] = 0.0;
      }
      const unsigned long long mk = __ballot(valid && rank == k - 1);
      const double kth = mk ? rl_f64(e, __builtin_ctzll(mk)) : -__builtin_huge_val();
      if (lane == 0) {
        ocnt[q] = cnt;
        const bool full = cid[base + kp - 1] >= 0;
        // an empty last slot with score +inf: the scan's list may be incomplete (k_pool_select)
        const bool trunc = !full && cs[base + kp - 1] == __builtin_huge_val();
        int res = trunc ? 0 : 1;
        if (full) {
          const double bound = cs[base + kp - 1] + eps;
          if (n >= k) res = k32 ? (float)bound < (float)kth : bound < kth;
          else if (thr_mode == 0) res = 0;
          else res = thr_mode == 1 ? (bound < thr_low(thr)) : (bound <= thr_low(thr));
        }
        ores[q] = res;
        if (oredo && (res == 0 || (count_empty && cnt == 0))) atomicAdd(oredo, 1);
      }
    }
    __syncthreads();
  }
}

// segments of <= 128 values: at most 128 VGPRs (4 waves per SIMD), so four workgroups per CU keep a
// 1000-query batch in one round (152 VGPRs allowed three per CU: 768 resident queries, the rest a second
// round of the whole latency chain)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_refine_lds_sm(HQ_REFINE_ARGS) {
  refine_lds_body<true>(HQ_REFINE_PASS);
}
// longer segments (out-of-line pairwise levels): the register-heavy general form
__global__ __launch_bounds__(256) void k_refine_lds(HQ_REFINE_ARGS) {
  refine_lds_body<false>(HQ_REFINE_PASS);
}

// ------------------------------------------------------------------------------------------------
// Long candidate lists (k > 64): the reference engine's default max_candidates_per_level = 100
// (core/search_engine.py:31, core/video_search.py:48) and SearchConfig's 1000 (config.py:181).  Same
// contracts as k_pool_select / k_refine_lds / k_progressive_final, one 256-thread workgroup per query,
// the orderings done as bitonic sorts in LDS instead of one entry per lane.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxTopKBig = 1024;  // list entries (k + slack) of the long-list path
constexpr int kSortCap = 4096;     // pool keys sorted whole in LDS (32 KiB); larger pools are cut first

__host__ __device__ __forceinline__ int pow2_at_least(int n) {
  int p = 2;
  while (p < n) p <<= 1;
  return p;
}

// ascending bitonic sort of n (a power of two) LDS entries; first(a, b): entry a ranks before entry b.
// All threads of the workgroup call it (the entries must be visible: a barrier before the call).
template <class First, class Swap>
__device__ __forceinline__ void lds_bitonic(int n, First first, Swap swp) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int size = 2; size <= n; size <<= 1)
    for (int st = size >> 1; st > 0; st >>= 1) {
      for (int t = tid; t < (n >> 1); t += nt) {
        const int lo = 2 * t - (t & (st - 1)), hi = lo + st;
        if (first(hi, lo) == ((lo & size) == 0)) swp(lo, hi);
      }
      __syncthreads();
    }
}

// Sort-based multi-stage select for long lists (k > 64).  The k-pass forms above (select_row, reg_topk)
// make k passes over every part: 0.74 s for one 1M-entry row at k = 1000.  Here stage 1 gives one
// 512-thread workgroup to each (query, part of <= kSortPart entries): the part's entries with their
// threshold test are sorted by (score desc, id asc) in LDS (bitonic; non-passing entries last) and its
// first k kept, plus the part's first arg-max over all its entries; each merge stage sorts the k-lists of
// kSortPart / k consecutive parts the same way, until one list per query remains.  The same total order
// and threshold test as select_row, so the result is identical.
constexpr int kSortPart = 4096;

__global__ __launch_bounds__(512) void k_select_sort(const double* __restrict__ in_s, const int64_t* __restrict__ in_id,
                                                     int Q, int64_t n_in, int64_t part, int P, int k, double thr,
                                                     int thr_mode, int final_stage, int64_t id_add,
                                                     double* __restrict__ o_s, int64_t* __restrict__ o_id,
                                                     double* __restrict__ o_b, int64_t* __restrict__ o_bid,
                                                     const double* __restrict__ i_b, const int64_t* __restrict__ i_bid,
                                                     int Pb) {
  __shared__ double ks[kSortPart];
  __shared__ int64_t ki[kSortPart];
  __shared__ double rb[8];
  __shared__ int64_t rbi[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool first_stage = in_id == nullptr;
  // (score, id) arg-max over the workgroup's threads (ids < 0: none)
  auto block_best = [&](double bs, int64_t bi, double& os, int64_t& oi) {
    for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bi, o, 64);
      if (i2 >= 0 && (bi < 0 || better(s2, i2, bs, bi))) { bs = s2; bi = i2; }
    }
    if (lane == 0) { rb[wave] = bs; rbi[wave] = bi; }
    __syncthreads();
    bs = rb[0];
    bi = rbi[0];
    for (int w = 1; w < 8; ++w)
      if (rbi[w] >= 0 && (bi < 0 || better(rb[w], rbi[w], bs, bi))) { bs = rb[w]; bi = rbi[w]; }
    __syncthreads();
    os = bs;
    oi = bi;
  };
  for (int64_t t = blockIdx.x; t < (int64_t)Q * P; t += gridDim.x) {
    const int64_t q = t / P, p = t % P;
    const int64_t c0 = p * part;
    const int n = (int)(c0 >= n_in ? 0 : (n_in - c0 < part ? n_in - c0 : part));
    const int n2 = pow2_at_least(n > 2 ? n : 2);
    double bs = 0.0;
    int64_t bi = -1;
    for (int x = tid; x < n2; x += 512) {
      double s = -__builtin_huge_val();
      int64_t id = -1;
      if (x < n) {
        s = in_s[q * n_in + c0 + x];
        if (first_stage) {
          id = c0 + x;
          if (bi < 0 || better(s, id, bs, bi)) { bs = s; bi = id; }  // first arg-max: every entry
          if (!(thr_mode == 0 || (thr_mode == 1 ? s >= thr : s > thr))) id = -1;
        } else {
          id = in_id[q * n_in + c0 + x];
        }
      }
      ks[x] = s;
      ki[x] = id;
    }
    double pbs;
    int64_t pbi;
    block_best(bs, bi, pbs, pbi);  // (its barrier also publishes ks / ki)
    lds_bitonic(n2,
                [&](int a, int b) {
                  const int64_t ia = ki[a], ib = ki[b];
                  return ia >= 0 && (ib < 0 || better(ks[a], ia, ks[b], ib));
                },
                [&](int a, int b) {
                  const double ts = ks[a];
                  ks[a] = ks[b];
                  ks[b] = ts;
                  const int64_t ti = ki[a];
                  ki[a] = ki[b];
                  ki[b] = ti;
                });
    for (int r = tid; r < k; r += 512) {
      const bool v = r < n && ki[r] >= 0;
      o_s[t * k + r] = v ? ks[r] : -__builtin_huge_val();
      o_id[t * k + r] = v ? ki[r] + (final_stage ? id_add : 0) : -1;
    }
    if (o_b) {
      if (first_stage) {
        if (tid == 0) {
          o_b[t] = pbi >= 0 ? pbs : -__builtin_huge_val();
          o_bid[t] = pbi >= 0 ? pbi + (final_stage ? id_add : 0) : -1;
        }
      } else if (final_stage) {  // the first arg-max of the query's stage-1 parts
        double cs = 0.0;
        int64_t ci = -1;
        for (int x = tid; x < Pb; x += 512) {
          const int64_t i = i_bid[q * Pb + x];
          if (i >= 0 && (ci < 0 || better(i_b[q * Pb + x], i, cs, ci))) { cs = i_b[q * Pb + x]; ci = i; }
        }
        double fs;
        int64_t fi;
        block_best(cs, ci, fs, fi);
        if (tid == 0) {
          o_b[q] = fi >= 0 ? fs : -__builtin_huge_val();
          o_bid[q] = fi >= 0 ? fi + id_add : -1;
        }
      }
    }
    __syncthreads();
  }
}

// pool entry -> 64-bit key, ascending = (score desc, row asc): scores are >= 0, so their f32 bit
// patterns order like the values; rows are unique within a pool, so keys are unique
__device__ __forceinline__ uint64_t pool_key(float s, int row) {
  return ((uint64_t)(0x7FFFFFFFu - __float_as_uint(s)) << 32) | (uint32_t)row;
}

// k_pool_select for K > 64.  A pool of T > K entries is first cut to exactly its K smallest keys by a radix
// select (8-bit digits from the top, a 256-bin LDS histogram per digit, stopping as soon as the K-th key's
// bucket is taken whole: 3-4 digits on scores of one exponent), reading a pool of <= kSortCap entries from
// LDS and a larger one from memory; only the K (<= kMaxTopKBig) survivors are sorted.  Round 4's form
// sorted the whole pool (2048-4096 keys at M = 1000: 78 bitonic stages of 8 swaps per thread) and cut larger
// pools by a 64-step bisection in memory.
// CAP: pool keys held in LDS, KC: list entries (K <= KC); <1024, 128> for M = 100 (10 KB of LDS: every
// workgroup of a 1000-query batch resident at once), <kSortCap, kMaxTopKBig> (41 KB) above
template <int CAP, int KC, int NT = 256>
__global__ __launch_bounds__(NT) void k_pool_sort(float* pool_s, int* pool_i, int* pool_n, int cap, int Q, int K,
                                                   int64_t id_base, double* __restrict__ out_score,
                                                   int64_t* __restrict__ out_id, const double* __restrict__ th0,
                                                   double thr0, const float* __restrict__ qflag, int qstride,
                                                   Scan0Args fa, const int* __restrict__ flist,
                                                   const int* __restrict__ fcount, int lds_cap) {
  __shared__ uint64_t key[CAP];
  __shared__ uint64_t sel[KC];
  __shared__ int hist[256];
  __shared__ int sb[3];  // the K-th key's bucket, the count before it, its count
  __shared__ int nsel;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    if (fcount) {  // the corpus's flagged rows against this query first (k_pool_select)
      const QConst* qc = reinterpret_cast<const QConst*>(fa.qconst);
      const int n = *fcount;
      if (n > 0 && __float_as_int(qc[q].flag) == 0) {
        const QConst c = qc[q];
        for (int i = tid; i < n; i += NT) flagged_pair(fa, c, q, flist[i]);
      }
      __syncthreads();
    }
    const int pn = fcount ? __hip_atomic_load(pool_n + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pool_n[q];
    if (qflag && (__float_as_int(qflag[(int64_t)q * qstride]) != 0 || pn > cap)) {
      for (int x = tid; x < K; x += NT) {
        out_score[(int64_t)q * K + x] = __builtin_huge_val();
        out_id[(int64_t)q * K + x] = -1;
      }
      continue;
    }
    const int T = pn < cap ? pn : cap;
    const float* ps = pool_s + (int64_t)q * cap;
    const int* pi = pool_i + (int64_t)q * cap;
    const int k = T < K ? T : K;
    const bool in_lds = T <= lds_cap && T <= CAP;
    if (T <= K) {
      for (int x = tid; x < T; x += NT) sel[x] = pool_key(ps[x], pi[x]);
    } else {
      if (in_lds)
        for (int x = tid; x < T; x += NT) key[x] = pool_key(ps[x], pi[x]);
      auto get = [&](int x) -> uint64_t { return in_lds ? key[x] : pool_key(ps[x], pi[x]); };
      uint64_t prefix = 0ull, mask = 0ull;
      int need = K;  // keys still to take among those matching prefix on mask
      for (int shift = 56; shift >= 0; shift -= 8) {
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int x = tid; x < T; x += NT) {
          const uint64_t kk = get(x);
          if ((kk & mask) == prefix) atomicAdd(&hist[(int)(kk >> shift) & 255], 1);
        }
        __syncthreads();
        if (wave == 0) {  // the bucket holding the need-th matching key
          const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
          int inc = h0 + h1 + h2 + h3;
          for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(inc, o, 64);
            if (lane >= o) inc += u;
          }
          int c = inc - (h0 + h1 + h2 + h3);
          const int hs[4] = {h0, h1, h2, h3};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (c < need && c + hs[j] >= need) { sb[0] = 4 * lane + j; sb[1] = c; sb[2] = hs[j]; }
            c += hs[j];
          }
        }
        __syncthreads();
        prefix |= (uint64_t)sb[0] << shift;
        mask |= 0xFFull << shift;
        need -= sb[1];
        const bool whole = sb[2] == need;
        __syncthreads();  // sb read by every thread before the next digit rewrites it
        if (whole) break;
      }
      // exactly K keys: those whose digits so far are <= the prefix's (keys are unique)
      if (tid == 0) nsel = 0;
      __syncthreads();
      for (int x = tid; x < T; x += NT) {
        const uint64_t kk = get(x);
        if ((kk & mask) <= prefix) sel[atomicAdd(&nsel, 1)] = kk;
      }
    }
    const int n2 = pow2_at_least(k);
    for (int x = k + tid; x < n2; x += NT) sel[x] = ~0ull;
    __syncthreads();
    lds_bitonic(n2, [&](int a, int b) { return sel[a] < sel[b]; },
                [&](int a, int b) { const uint64_t t = sel[a]; sel[a] = sel[b]; sel[b] = t; });
    const bool trunc = th0 != nullptr && th0[q] > thr0;
    for (int x = tid; x < K; x += NT) {
      if (x < k) {
        const uint64_t kk = sel[x];
        out_score[(int64_t)q * K + x] = (double)__uint_as_float(0x7FFFFFFFu - (uint32_t)(kk >> 32));
        out_id[(int64_t)q * K + x] = (int64_t)(uint32_t)kk + id_base;
      } else {
        out_score[(int64_t)q * K + x] = trunc ? __builtin_huge_val() : -__builtin_huge_val();
        out_id[(int64_t)q * K + x] = -1;
      }
    }
    __syncthreads();
  }
}

// pool select launcher: one wave per query up to 64 entries, the LDS sort above beyond
static void launch_pool_select(int K, hipStream_t s, int Q, float* pool_s, int* pool_i, int* pool_n, int cap,
                               int64_t id_base, double* out_score, int64_t* out_id, const double* th0, double thr0,
                               const float* qflag, int qstride, const Scan0Args& fa, const int* flist,
                               const int* fcount) {
  const int mg = Q < 8192 ? Q : 8192;
  if (K <= kMaxTopK)
    hipLaunchKernelGGL(k_pool_select, dim3(mg), dim3(64), 0, s, pool_s, pool_i, pool_n, cap, Q, K, id_base, out_score,
                       out_id, th0, thr0, qflag, qstride, fa, flist, fcount);
  else if (K <= 128)
    hipLaunchKernelGGL((k_pool_sort<1024, 128>), dim3(mg), dim3(256), 0, s, pool_s, pool_i, pool_n, cap, Q, K, id_base,
                       out_score, out_id, th0, thr0, qflag, qstride, fa, flist, fcount,
                       opt(OPT_POOL_SORT_MEM, 0) ? 0 : 1024);  // option pool_sort_mem: test the memory form
  else
    hipLaunchKernelGGL((k_pool_sort<kSortCap, kMaxTopKBig, 512>), dim3(mg), dim3(512), 0, s, pool_s, pool_i, pool_n, cap, Q,
                       K, id_base, out_score, out_id, th0, thr0, qflag, qstride, fa, flist, fcount,
                       opt(OPT_POOL_SORT_MEM, 0) ? 0 : kSortCap);
}

// k_refine_lds for kp > 64 (same contract, arithmetic and outputs), one 256-thread workgroup per query.
// Pass 1: each thread scores list entries tid, tid + 256, ... straight from global memory (the level the
// ranking needs: level 0 in mode 0, the overall in mode 1) — a round's 256 row reads are independent, so
// they are all in flight — and keeps (score, id) in LDS; a bitonic sort ranks them (score desc, id asc).
// Pass 2 (odet): one thread per output entry computes its [overall, level..] record (exact_pair writes the
// levels into the record directly).  The LDS-staged form of round 4's first version (tiles of rows, one
// level task per thread) spent most of its time in the staging round trips: 111 us at M = 100, 923 us at
// M = 1000 per 1000-query batch.
// ZB: the candidates' normalised values from Z (true) or recomputed from their raw rows (false: half the
// bytes, an f64 division per value; A/B per 1000-query batch: M = 1000 896 -> 746 us, M = 100 116 -> 129).
// The raw form sums the correlation and the squared differences in one pass over the row (F2: each row
// value loaded once; k_refine_big_sm_raw 771 -> 608 us at M = 1000, no scratch); the Z form keeps two
// passes (F2 there: 248 VGPRs + scratch, M = 100 4% slower)
template <bool SM, bool ZB = true>
__device__ __forceinline__ void refine_big_body(HQ_REFINE_ARGS, int tb) {
  if (onext && blockIdx.x == 0 && threadIdx.x == 0) *onext = 0;  // the next batch's redo counter
  __shared__ double se[kMaxTopKBig];
  __shared__ int64_t sid[kMaxTopKBig];
  __shared__ int red[4];
  (void)tb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W = 1 + si.nseg;
  const int n2 = pow2_at_least(kp);
  const bool k32 = (thr_mode & kThrKey32) != 0;
  thr_mode &= kThrKey32 - 1;
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    const int64_t base = (int64_t)q * kp;
    // ---- pass 1: exact ranking score of every list entry ----
    int nv = 0;
    for (int x = tid; x < n2; x += 256) {
      double e = -__builtin_huge_val();
      int64_t id = -1;
      if (x < kp) {
        const int64_t cid_x = cid[base + x];
        const int64_t c = cid_x - id_base;
        if (cid_x >= 0 && c >= 0 && c < N) {
          int typed = 0;
          const double v = exact_pair<SM, ZB, !ZB>(Qs, q, Cs, c, si, mode == 0 ? 0 : -1, nullptr, &typed);
          const bool pass = mode == 0 ? typed_pass(v, typed, thr, thr_mode)
                                      : (thr_mode == 0 || (thr_mode == 1 ? v >= thr : v > thr));
          if (pass) {
            e = v;
            id = cid_x;
            ++nv;
          }
        }
      }
      se[x] = e;
      sid[x] = id;
    }
    nv = wsum64i(nv);
    if (lane == 0) red[wave] = nv;
    __syncthreads();
    const int n = red[0] + red[1] + red[2] + red[3];
    // ---- rank: (score desc, id asc), invalid entries last ----
    lds_bitonic(n2,
                [&](int a, int b) {
                  const int64_t ia = sid[a], ib = sid[b];
                  if (ib < 0) return ia >= 0;
                  const double ka = key_of(se[a], k32), kb = key_of(se[b], k32);
                  return ia >= 0 && (ka > kb || (ka == kb && ia < ib));
                },
                [&](int a, int b) {
                  const double te = se[a];
                  se[a] = se[b];
                  se[b] = te;
                  const int64_t ti = sid[a];
                  sid[a] = sid[b];
                  sid[b] = ti;
                });
    const int cnt = n < k ? n : k;
    for (int x = tid; x < k; x += 256) {
      os[(int64_t)q * k + x] = x < cnt ? se[x] : -__builtin_huge_val();
      oid[(int64_t)q * k + x] = x < cnt ? sid[x] : -1;
      if (odet) {
        double* rec = odet + ((int64_t)q * k + x) * W;
        if (x < cnt) {
          // ---- pass 2: the output entry's [overall, level..] record ----
          rec[0] = exact_pair<SM, ZB, !ZB>(Qs, q, Cs, sid[x] - id_base, si, -1, rec + 1);
        } else {
          for (int w = 0; w < W; ++w) rec[w] = 0.0;
        }
      }
    }
    if (tid == 0) {
      const double kth = n >= k ? se[k - 1] : -__builtin_huge_val();
      ocnt[q] = cnt;
      const bool full = cid[base + kp - 1] >= 0;
      // an empty last slot with score +inf: the scan's list may be incomplete (k_pool_select)
      const bool trunc = !full && cs[base + kp - 1] == __builtin_huge_val();
      int res = trunc ? 0 : 1;
      if (full) {
        const double bound = cs[base + kp - 1] + eps;
        if (n >= k) res = k32 ? (float)bound < (float)kth : bound < kth;
        else if (thr_mode == 0) res = 0;
        else res = thr_mode == 1 ? (bound < thr_low(thr)) : (bound <= thr_low(thr));
      }
      ores[q] = res;
      if (oredo && (res == 0 || (count_empty && cnt == 0))) atomicAdd(oredo, 1);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_refine_big_sm(HQ_REFINE_ARGS, int tb) { refine_big_body<true>(HQ_REFINE_PASS, tb); }
__global__ __launch_bounds__(256) void k_refine_big(HQ_REFINE_ARGS, int tb) { refine_big_body<false>(HQ_REFINE_PASS, tb); }
__global__ __launch_bounds__(256) void k_refine_big_sm_raw(HQ_REFINE_ARGS, int tb) {
  refine_big_body<true, false>(HQ_REFINE_PASS, tb);
}
__global__ __launch_bounds__(256) void k_refine_big_raw(HQ_REFINE_ARGS, int tb) {
  refine_big_body<false, false>(HQ_REFINE_PASS, tb);
}

// ------------------------------------------------------------------------------------------------
// Lane-cooperative long-list re-rank (kp > 64, every level segment <= 128 values, L <= 128 even): the
// default for the reference's M = 100 / 1000 lists.  k_refine_big gives each list entry one thread that
// walks its candidate row 8 bytes at a time (a wave load instruction touches 64 rows: ~115 L2 requests
// per pair, 79% of the wave cycles waiting on memory).  Here a group of 8 lanes scores one entry:
//  * the group stages the candidate's raw row and statistics into its own LDS buffer with 16-byte loads
//    (one wave load instruction = 8 rows x 128 contiguous bytes), one entry ahead in registers;
//  * every NumPy pairwise sum of the exact score (n <= 128: eight strided accumulators r_j += a[i + j],
//    ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), a sequential tail) runs with lane j owning r_j; the combination
//    is three xor-shuffle adds (IEEE addition is commutative: both partners hold the same bits), the tail
//    and the sums of < 8 values are evaluated identically by all 8 lanes — bit-identical to np_sum;
//  * one pass computes every level of the entry (the [overall, level..] record), so each row is gathered
//    once (k_refine_big: level 0 for the ranking, then the whole row again for the record).  Records of
//    entries x < k go to odet[q][x] unsorted, the slack entries' to LDS; after the (score desc, id asc)
//    bitonic sort every thread reads its outputs' records into registers (L1-bypassing loads), a
//    barrier, then writes them in sorted order.
// ------------------------------------------------------------------------------------------------
// 1 / (level + 1) of the overall score's weights (search_engine.py:191-230), folded at compile time
__device__ constexpr double kLevelWeight[8] = {1.0 / 1.0, 1.0 / 2.0, 1.0 / 3.0, 1.0 / 4.0, 1.0 / 5.0, 1.0 / 6.0, 1.0 / 7.0, 1.0 / 8.0};
constexpr int kFinalRounds = 32;  // final rankings of <= 32 outputs may take arg-max rounds instead of a sort
constexpr int kCoopGroups = 32;              // 8-lane groups per 256-thread workgroup
constexpr int kCoopMaxW = 7;                 // record width 1 + nseg

// the group partner's value by DPP (a VALU operand modifier; __shfl_xor goes through the LDS crossbar,
// ds_bpermute, three dependent round trips per sum): M = 1, 2 quad_perm [1,0,3,2] / [2,3,0,1]; M = 4
// row_half_mirror (lane i of 8 reads lane 7 - i: after the first two steps lanes 0-3 hold the same bits and
// so do lanes 4-7, so any cross pairing gives the same sum)
template <int M>
__device__ __forceinline__ int coop_dpp(int v) {
  constexpr int ctrl = M == 1 ? 0xB1 : (M == 2 ? 0x4E : 0x141);
  return __builtin_amdgcn_update_dpp(v, v, ctrl, 0xF, 0xF, false);
}
template <int M>
__device__ __forceinline__ float coop_xor(float v) { return __int_as_float(coop_dpp<M>(__float_as_int(v))); }
template <int M>
__device__ __forceinline__ double coop_xor(double v) {
  const int lo = coop_dpp<M>(__double2loint(v)), hi = coop_dpp<M>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int M, typename T>
__device__ __forceinline__ Sum2<T> coop_xor(Sum2<T> v) {
  return Sum2<T>(coop_xor<M>(v.a), coop_xor<M>(v.b));
}

// np_sum<T, true>(f, n) (n <= 128) over the 8 lanes of a group; j = lane within the group.  Every lane
// returns the same bits.
template <typename T, class F>
__device__ __forceinline__ T coop_sum(const F& f, int n, int j) {
  T res;
  if (n < 8) {
    res = T(-0.0);
#pragma unroll 1
    for (int i = 0; i < n; ++i) res = res + f(i);
  } else {
    T r = f(j);
    const int lim = n - (n % 8);
#pragma unroll 1
    for (int i = 8 + j; i < lim; i += 8) r = r + f(i);
    r = r + coop_xor<1>(r);  // r_j + r_(j^1): (r0 + r1) on lanes 0 and 1
    r = r + coop_xor<2>(r);  // (r0 + r1) + (r2 + r3)
    r = r + coop_xor<4>(r);  // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
    res = r;
#pragma unroll 1
    for (int i = lim; i < n; ++i) res = res + f(i);
  }
  return T(0) + res;
}

// make_side<true> with the float32 statistics summed by the group
__device__ __forceinline__ Side coop_side(const double* x, const double* z, const double* st, int m, bool f32, int j) {
  Side r;
  r.x = x;
  r.z = z;
  r.f32 = f32;
  if (f32) {
    auto gx = [=](int k) -> float { return (float)x[k]; };
    const float mean = coop_sum<float>(gx, m, j) / (float)m;
    auto gd = [=](int k) -> float { const float d = (float)x[k] - mean; return d * d; };
    const float sd = sqrtf(coop_sum<float>(gd, m, j) / (float)m);
    auto gs = [=](int k) -> float { const float v = (float)x[k]; return v * v; };
    r.mean = mean;
    r.sd = sd;
    r.msq = coop_sum<float>(gs, m, j) / (float)m;
  } else {
    r.mean = st[0];
    r.sd = st[1];
    r.msq = st[2];
  }
  return r;
}

// exact_level_sides<true, true> (one-pass Sum2 form) with the sums over the group
__device__ __forceinline__ double coop_level_sides(const Side& q, const Side& c, int m, int j, int* np32) {
  *np32 = 0;
  const bool both32 = q.f32 && c.f32;
  if (q.sd == 0.0 || c.sd == 0.0) return const0(q.sd == 0.0, c.sd == 0.0, q.mean, c.mean, both32);  // :141-148
  if (both32) {
    auto f2 = [&](int k) -> Sum2<float> {
      const float d = (float)q.x[k] - (float)c.x[k];
      return Sum2<float>((float)side_z(q, k) * (float)side_z(c, k), d * d);
    };
    const Sum2<float> s2 = coop_sum<Sum2<float>>(f2, m, j);
    const float corr = s2.a / (float)m;                                            // :154
    const float mse = s2.b / (float)m;                                             // :161
    const float sim = (corr + 1.0f) / 2.0f;                                        // :158
    const float maxmse = (float)q.msq + (float)c.msq;                              // :162
    float ds = 1.0f;
    if (maxmse > 0.0f) {
      ds = 1.0f - mse / maxmse;
      ds = ds > 0.0f ? ds : 0.0f;
    }
    const float comb = 0.7f * sim + 0.3f * ds;                                     // :171
    if (comb < 1.0f && comb > 0.0f) {
      *np32 = 1;
      return comb;
    }
    return comb < 1.0f ? 0.0 : 1.0;                                                // :174
  }
  auto f2 = [&](int k) -> Sum2<double> {
    const double d = q.x[k] - c.x[k];
    return Sum2<double>(side_z(q, k) * side_z(c, k), d * d);
  };
  const Sum2<double> s2 = coop_sum<Sum2<double>>(f2, m, j);
  const double corr = s2.a / (double)m;                                            // :154
  const double mse = s2.b / (double)m;                                             // :161
  const double sim = (corr + 1.0) / 2.0;                                           // :158
  const double maxmse = q.msq + c.msq;                                             // :162
  double ds = 1.0;
  if (maxmse > 0.0) {
    ds = 1.0 - (mse / maxmse);
    ds = ds > 0.0 ? ds : 0.0;
  }
  const double a = 0.7 * sim;
  const double b = 0.3 * ds;
  double comb = a + b;                                                             // :171
  comb = comb < 1.0 ? comb : 1.0;
  return comb > 0.0 ? comb : 0.0;
}

// coop_level_sides in two phases, so that the scalar tail of a level (divisions, clamps) runs once per
// group instead of on all 8 lanes: the sums (all lanes, group-cooperative; kind 0 = a zero-variance side,
// no sums; 1 = float32 sums; 2 = float64 sums), then level_finish on the lane that owns the level.
struct LevelStat {
  double qm, qs, qq, cm, cs, cq;  // both sides' mean, std, mean of squares (their own dtype's values)
  double sa, sb;                  // the correlation products' and squared differences' sums
  int kind, both32;
};
__device__ __forceinline__ LevelStat coop_level_sums(const Side& q, const Side& c, int m, int j) {
  LevelStat r;
  r.qm = q.mean; r.qs = q.sd; r.qq = q.msq;
  r.cm = c.mean; r.cs = c.sd; r.cq = c.msq;
  r.both32 = q.f32 && c.f32;
  r.sa = 0.0;
  r.sb = 0.0;
  if (q.sd == 0.0 || c.sd == 0.0) {
    r.kind = 0;
  } else if (r.both32) {
    auto f2 = [&](int k) -> Sum2<float> {
      const float d = (float)q.x[k] - (float)c.x[k];
      return Sum2<float>((float)side_z(q, k) * (float)side_z(c, k), d * d);
    };
    const Sum2<float> s2 = coop_sum<Sum2<float>>(f2, m, j);
    r.sa = s2.a;
    r.sb = s2.b;
    r.kind = 1;
  } else {
    auto f2 = [&](int k) -> Sum2<double> {
      const double d = q.x[k] - c.x[k];
      return Sum2<double>(side_z(q, k) * side_z(c, k), d * d);
    };
    const Sum2<double> s2 = coop_sum<Sum2<double>>(f2, m, j);
    r.sa = s2.a;
    r.sb = s2.b;
    r.kind = 2;
  }
  return r;
}
// the tail of coop_level_sides from its sums (the same expressions, the same result bits)
__device__ __forceinline__ double level_finish(const LevelStat& t, int m, int* np32) {
  *np32 = 0;
  if (t.kind == 0) return const0(t.qs == 0.0, t.cs == 0.0, t.qm, t.cm, t.both32 != 0);  // :141-148
  if (t.kind == 1) {
    const float corr = (float)t.sa / (float)m;                                     // :154
    const float mse = (float)t.sb / (float)m;                                      // :161
    const float sim = (corr + 1.0f) / 2.0f;                                        // :158
    const float maxmse = (float)t.qq + (float)t.cq;                                // :162
    float ds = 1.0f;
    if (maxmse > 0.0f) {
      ds = 1.0f - mse / maxmse;
      ds = ds > 0.0f ? ds : 0.0f;
    }
    const float comb = 0.7f * sim + 0.3f * ds;                                     // :171
    if (comb < 1.0f && comb > 0.0f) {
      *np32 = 1;
      return comb;
    }
    return comb < 1.0f ? 0.0 : 1.0;                                                // :174
  }
  const double corr = t.sa / (double)m;                                            // :154
  const double mse = t.sb / (double)m;                                             // :161
  const double sim = (corr + 1.0) / 2.0;                                           // :158
  const double maxmse = t.qq + t.cq;                                               // :162
  double ds = 1.0;
  if (maxmse > 0.0) {
    ds = 1.0 - (mse / maxmse);
    ds = ds > 0.0 ? ds : 0.0;
  }
  const double a = 0.7 * sim;
  const double b = 0.3 * ds;
  double comb = a + b;                                                             // :171
  comb = comb < 1.0 ? comb : 1.0;
  return comb > 0.0 ? comb : 0.0;
}

// Compact level table of the cooperative kernels (a full SegInfo by value costs SGPRs they need)
struct CoopSeg {
  int nseg, L, Lp;
  int src[kCoopMaxW - 1], len[kCoopMaxW - 1], poff[kCoopMaxW - 1];
};

// k_rank_pairs + k_rank_sort arguments; workspace per list entry: score (f64), id (i64) and, with records,
// the [overall, level..] record (W doubles)
struct RankArgs {
  const double* Rq; const double* Zq; const double* Sq; int Q;
  const double* Rc; const double* Sc; int64_t N;
  CoopSeg cs;
  int mode, kp, k, thr_mode, det;
  double thr;
  int64_t id_base;
  const int64_t* cid;
  double* ws_sc; int64_t* ws_id; double* ws_rec;
  int win;  // k_rank_sort: window ranking before the bitonic sort (option rank_win, default 1)
};

__host__ __device__ inline int coop_qw(const CoopSeg& c) { return (c.L + c.Lp + 4 * c.nseg + 1) & ~1; }
// (>= 12: after scoring, a group's buffer carries its 8 level values and flags, k_rank_pairs)
__host__ __device__ inline int coop_rw(const CoopSeg& c) {
  const int w = (c.L + 4 * c.nseg + 1) & ~1;
  return w > 12 ? w : 12;
}

// Scoring pass: block (x-block, query) = 32 list entries of one query, one 8-lane group per entry.  The
// block stages the query row (raw, Z, S) and each group its candidate's raw row and statistics (16-byte
// loads: one wave load instruction covers 8 rows x 128 contiguous bytes) into LDS, then the group scores
// every level of the entry (nlev: level 0 only for a mode-0 ranking without records) and writes the
// ranking score, id and record to the workspace.  One pair per group, no loop: the occupancy hides the
// row latency.  Bit-identical to exact_pair (coop_level_sides = exact_level_sides<true, true>).
// the query row (raw, Z, S: all NT threads of the block) and, for list entry x < kp, group g's candidate row
// and statistics (16-byte loads) into LDS; returns the candidate's local row (-1: none)
template <int PPL>
__device__ __forceinline__ int64_t rank_stage(const RankArgs& a, double* rq, double* rg, int q, int x, int tid, int nt,
                                              int j) {
  const int L = a.cs.L, Lp = a.cs.Lp, nseg = a.cs.nseg;
  // the query row, normalised row and statistics (QW = L + Lp + 4 nseg values; one value per thread when
  // QW <= nt, the cooperative shapes' case) and this group's list entry are requested together: one round trip
  // before the candidate's row (loop-per-array stores waited for each array in turn: 4 round trips)
  const int QW = L + Lp + 4 * nseg;
  const int64_t idr = x < a.kp ? a.cid[(int64_t)q * a.kp + x] : -1;
  if (QW <= nt) {
    if (tid < QW) {
      const double* src = tid < L ? a.Rq + (int64_t)q * L + tid
                        : tid < L + Lp ? a.Zq + (int64_t)q * Lp + (tid - L)
                                       : a.Sq + (int64_t)q * nseg * 4 + (tid - L - Lp);
      rq[tid] = *src;
    }
  } else {
    for (int e = tid; e < L; e += nt) rq[e] = a.Rq[(int64_t)q * L + e];
    for (int e = tid; e < Lp; e += nt) rq[L + e] = a.Zq[(int64_t)q * Lp + e];
    for (int e = tid; e < 4 * nseg; e += nt) rq[L + Lp + e] = a.Sq[(int64_t)q * nseg * 4 + e];
  }
  int64_t c = -1;
  if (x < a.kp) {
    const int64_t cc = idr - a.id_base;
    if (idr >= 0 && cc >= 0 && cc < a.N) c = cc;
  }
  if (c >= 0) {
    const int np_raw = L / 2, np_all = np_raw + 2 * nseg;
    const f64x2* rr = reinterpret_cast<const f64x2*>(a.Rc + c * L);
    const f64x2* rs = reinterpret_cast<const f64x2*>(a.Sc + c * nseg * 4);
    // every piece loaded before the first LDS store (unconditional loads of a clamped piece: a conditionally
    // filled register array was merged into one 24-register tuple and spilled)
    f64x2 v[PPL];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
      const int pc = j + 8 * p < np_all ? j + 8 * p : np_all - 1;
      v[p] = *(pc < np_raw ? rr + pc : rs + (pc - np_raw));
    }
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
      const int pc = j + 8 * p;
      if (pc < np_all) reinterpret_cast<f64x2*>(rg)[pc] = v[p];
    }
  }
  return c;
}

// one list entry scored by its 8-lane group (staged rows: rank_stage): the ranking score e and id (-inf / -1
// when it fails the threshold or has no row) and, with a.det, its [overall, level..] record in rec[0 .. W)
// (lane j writes level j).  Every level's sums are group-cooperative; lane j keeps level j's and finishes it
// alone (the scalar tail of a level runs once per group, not on all 8 lanes); the levels' values reach every
// lane of the group through its row buffer (the rows are consumed by then).  Bit-identical to exact_pair.
__device__ __forceinline__ void rank_score(const RankArgs& a, const double* rq, double* rg, int64_t c, int j,
                                           double* rec, double& e, int64_t& id) {
  const int L = a.cs.L, Lp = a.cs.Lp, nseg = a.cs.nseg;
  e = -__builtin_huge_val();
  id = -1;
  if (c < 0) return;
  const int nlev = (a.mode == 0 && !a.det) ? 1 : nseg;
  LevelStat mine;
  mine.kind = 0; mine.both32 = 0;
  mine.qm = mine.qs = mine.qq = mine.cm = mine.cs = mine.cq = mine.sa = mine.sb = 0.0;
#pragma unroll 1
  for (int s = 0; s < nlev; ++s) {
    const int m = a.cs.len[s];
    const double* qst = rq + L + Lp + 4 * s;
    const double* cst = rg + L + 4 * s;
    const LevelStat t = coop_level_sums(
        coop_side(rq + a.cs.src[s], rq + L + a.cs.poff[s], qst, m, (aux_bits(qst) & kAuxF32) != 0, j),
        coop_side(rg + a.cs.src[s], nullptr, cst, m, (aux_bits(cst) & kAuxF32) != 0, j), m, j);
    if (j == s) mine = t;
  }
  int t32 = 0;
  const double vj = j < nlev ? level_finish(mine, a.cs.len[j < nlev ? j : 0], &t32) : 0.0;
  if (a.det && j < nlev) rec[1 + j] = vj;
  wave_lds_sync();
  if (j < nlev) {
    rg[j] = vj;
    reinterpret_cast<int*>(rg + 8)[j] = t32;
  }
  wave_lds_sync();
  const double v0 = rg[0];
  const int t0 = reinterpret_cast<const int*>(rg + 8)[0];
  double tws = 0.0, tw = 0.0;
  bool acc32 = false;
#pragma unroll 1
  for (int s = 0; s < nlev; ++s) {
    // search_engine.py:191-230 typed running sum (exact_pair_rows)
    const double v = rg[s];
    const int ts = reinterpret_cast<const int*>(rg + 8)[s];
    const double w = kLevelWeight[s];
    const double term = ts ? (double)((float)v * (float)w) : v * w;
    if (!acc32 && !ts) {
      tws = tws + term;
    } else {
      tws = (double)((float)tws + (float)term);
      acc32 = true;
    }
    tw = tw + w;
  }
  double ov = 0.0;
  if (nlev == nseg) {
    if (acc32) {
      const float o = (float)tws / (float)tw;
      ov = o < 1.0f ? (double)o : 1.0;
    } else {
      ov = tw > 0.0 ? tws / tw : 0.0;
      ov = ov < 1.0 ? ov : 1.0;
    }
    ov = ov > 0.0 ? ov : 0.0;
  }
  if (a.det && j == 0) rec[0] = ov;
  const double v = a.mode == 0 ? v0 : ov;
  const int tm = a.thr_mode & (kThrKey32 - 1);  // the test itself (kThrKey32: the sort keys only)
  const bool pass = a.mode == 0 ? typed_pass(v, t0, a.thr, tm) : (tm == 0 || (tm == 1 ? v >= a.thr : v > a.thr));
  if (pass) {
    e = v;
    id = c + a.id_base;
  }
}

// ---- compile-time level structures of the cooperative scorers (LID 1: L = 64, 2: L = 32; 0: runtime) ----
// With the structure known, every level loop and every pairwise sum unrolls: the per-level trip counts,
// the n < 8 branches and the LDS offsets of each level become constants (k_rank_pairs' PMC, r05: 504 SALU
// per wave, mostly the runtime loops over levels and values).  The arithmetic and its order are rank_score's.
template <int LID> struct CoopT;
template <> struct CoopT<1> {  // L = 64: levels [0, 32) [32, 40) [40, 43) [43, 44) [44, 64), Lp = 68
  static constexpr int L = 64, Lp = 68, NSEG = 5;
  static constexpr int len(int s) { return s == 0 ? 32 : s == 1 ? 8 : s == 2 ? 3 : s == 3 ? 1 : 20; }
  static constexpr int src(int s) { return s == 0 ? 0 : s == 1 ? 32 : s == 2 ? 40 : s == 3 ? 43 : 44; }
  static constexpr int poff(int s) { return s == 0 ? 0 : s == 1 ? 32 : s == 2 ? 40 : s == 3 ? 44 : 48; }
};
template <> struct CoopT<2> {  // L = 32: levels [0, 16) [16, 20) [20, 21) [21, 32), Lp = 36
  static constexpr int L = 32, Lp = 36, NSEG = 4;
  static constexpr int len(int s) { return s == 0 ? 16 : s == 1 ? 4 : s == 2 ? 1 : 11; }
  static constexpr int src(int s) { return s == 0 ? 0 : s == 1 ? 16 : s == 2 ? 20 : 21; }
  static constexpr int poff(int s) { return s == 0 ? 0 : s == 1 ? 16 : s == 2 ? 20 : 24; }
};
// the LID whose table equals the runtime structure, else 0
static int coop_lid(const CoopSeg& c) {
  auto same = [&](auto t) {
    using T = decltype(t);
    if (c.L != T::L || c.Lp != T::Lp || c.nseg != T::NSEG) return false;
    for (int s = 0; s < T::NSEG; ++s)
      if (c.len[s] != T::len(s) || c.src[s] != T::src(s) || c.poff[s] != T::poff(s)) return false;
    return true;
  };
  if (opt(OPT_RANK_CT, 1) == 0) return 0;  // option rank_ct 0: the runtime-structure scorer (A/B, parity)
  // (rank_ct 2: also in the short-list kernel k_rank_small)
  if (same(CoopT<1>{})) return 1;
  if (same(CoopT<2>{})) return 2;
  return 0;
}

// coop_sum with n known at compile time (every loop unrolled; the same additions in the same order)
template <typename T, int N, class F>
__device__ __forceinline__ T coop_sum_n(const F& f, int j) {
  T res;
  if constexpr (N < 8) {
    res = T(-0.0);
#pragma unroll
    for (int i = 0; i < N; ++i) res = res + f(i);
  } else {
    constexpr int LIM = N - (N % 8);
    T r = f(j);
#pragma unroll
    for (int t = 1; t < LIM / 8; ++t) r = r + f(8 * t + j);
    r = r + coop_xor<1>(r);
    r = r + coop_xor<2>(r);
    r = r + coop_xor<4>(r);
    res = r;
#pragma unroll
    for (int i = LIM; i < N; ++i) res = res + f(i);
  }
  return T(0) + res;
}

// coop_level_sums for a level of M values (float64 sides: the candidate's z recomputed as (x - mean) / std;
// float32 sides keep the runtime form)
template <int M>
__device__ __forceinline__ LevelStat coop_level_sums_n(const Side& q, const Side& c, int j) {
  if (q.f32 || c.f32) return coop_level_sums(q, c, M, j);
  LevelStat r;
  r.qm = q.mean; r.qs = q.sd; r.qq = q.msq;
  r.cm = c.mean; r.cs = c.sd; r.cq = c.msq;
  r.both32 = 0;
  r.sa = 0.0;
  r.sb = 0.0;
  if (q.sd == 0.0 || c.sd == 0.0) {
    r.kind = 0;
  } else {
    auto f2 = [&](int k) -> Sum2<double> {
      const double d = q.x[k] - c.x[k];
      return Sum2<double>(side_z(q, k) * side_z(c, k), d * d);
    };
    const Sum2<double> s2 = coop_sum_n<Sum2<double>, M>(f2, j);
    r.sa = s2.a;
    r.sb = s2.b;
    r.kind = 2;
  }
  return r;
}

// rank_score with the level structure of CoopT<LID> (LID > 0) — the same values, bit for bit
template <int LID>
__device__ __forceinline__ void rank_score_t(const RankArgs& a, const double* rq, double* rg, int64_t c, int j,
                                             double* rec, double& e, int64_t& id) {
  if constexpr (LID == 0) {
    rank_score(a, rq, rg, c, j, rec, e, id);
  } else {
    using T = CoopT<LID>;
    constexpr int L = T::L, Lp = T::Lp, NS = T::NSEG;
    e = -__builtin_huge_val();
    id = -1;
    if (c < 0) return;
    const bool all = !(a.mode == 0 && !a.det);  // every level (records / overall ranking), else level 0 only
    LevelStat mine;
    mine.kind = 0; mine.both32 = 0;
    mine.qm = mine.qs = mine.qq = mine.cm = mine.cs = mine.cq = mine.sa = mine.sb = 0.0;
    auto level = [&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int m = T::len(s);
      const double* qst = rq + L + Lp + 4 * s;
      const double* cst = rg + L + 4 * s;
      const LevelStat t = coop_level_sums_n<m>(
          coop_side(rq + T::src(s), rq + L + T::poff(s), qst, m, (aux_bits(qst) & kAuxF32) != 0, j),
          coop_side(rg + T::src(s), nullptr, cst, m, (aux_bits(cst) & kAuxF32) != 0, j), j);
      if (j == s) mine = t;
    };
    level(std::integral_constant<int, 0>{});
    if (all) {
      level(std::integral_constant<int, 1>{});
      level(std::integral_constant<int, 2>{});
      level(std::integral_constant<int, 3>{});
      if constexpr (NS > 4) level(std::integral_constant<int, 4>{});
    }
    const int nlev = all ? NS : 1;
    int t32 = 0;
    int mj = T::len(0);
#pragma unroll
    for (int s = 1; s < NS; ++s) mj = j == s ? T::len(s) : mj;
    const double vj = j < nlev ? level_finish(mine, mj, &t32) : 0.0;
    if (a.det && j < nlev) rec[1 + j] = vj;
    wave_lds_sync();
    if (j < nlev) {
      rg[j] = vj;
      reinterpret_cast<int*>(rg + 8)[j] = t32;
    }
    wave_lds_sync();
    const double v0 = rg[0];
    const int t0 = reinterpret_cast<const int*>(rg + 8)[0];
    double ov = 0.0;
    if (all) {
      double tws = 0.0, tw = 0.0;
      bool acc32 = false;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        // search_engine.py:191-230 typed running sum (exact_pair_rows)
        const double v = rg[s];
        const int ts = reinterpret_cast<const int*>(rg + 8)[s];
        const double w = kLevelWeight[s];
        const double term = ts ? (double)((float)v * (float)w) : v * w;
        if (!acc32 && !ts) {
          tws = tws + term;
        } else {
          tws = (double)((float)tws + (float)term);
          acc32 = true;
        }
        tw = tw + w;
      }
      if (acc32) {
        const float o = (float)tws / (float)tw;
        ov = o < 1.0f ? (double)o : 1.0;
      } else {
        ov = tw > 0.0 ? tws / tw : 0.0;
        ov = ov < 1.0 ? ov : 1.0;
      }
      ov = ov > 0.0 ? ov : 0.0;
    }
    if (a.det && j == 0) rec[0] = ov;
    const double v = a.mode == 0 ? v0 : ov;
    const int tm = a.thr_mode & (kThrKey32 - 1);
    const bool pass = a.mode == 0 ? typed_pass(v, t0, a.thr, tm) : (tm == 0 || (tm == 1 ? v >= a.thr : v > a.thr));
    if (pass) {
      e = v;
      id = c + a.id_base;
    }
  }
}

// Scoring pass: block (x-block, query) = 32 list entries of one query, one 8-lane group per entry, scores
// and records to the workspace.  One pair per group, no loop: the occupancy hides the row latency.
template <int PPL, int LID = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LID == 2 ? 6 : 5))) void k_rank_pairs(RankArgs a) {
  extern __shared__ __attribute__((aligned(16))) double cm[];
  const int tid = threadIdx.x, g = tid >> 3, j = tid & 7;
  const int q = blockIdx.y, x = blockIdx.x * kCoopGroups + g;
  double* rq = cm;
  double* rg = cm + coop_qw(a.cs) + g * coop_rw(a.cs);
  const int64_t c = rank_stage<PPL>(a, rq, rg, q, x, tid, 256, j);
  __syncthreads();
  if (x >= a.kp) return;
  const int64_t e0 = (int64_t)q * a.kp + x;
  double e;
  int64_t id;
  rank_score_t<LID>(a, rq, rg, c, j, a.ws_rec + e0 * (1 + a.cs.nseg), e, id);
  if (j == 0) {
    a.ws_sc[e0] = e;
    a.ws_id[e0] = id;
  }
}

// the count and the completeness proof of query q's re-ranked list (refine_big_body): n valid entries, kth
// the k-th exact score (-inf when n < k); the last list slot's approximate score + eps must stay below it
// last_id / last_cs: the list's last slot (cid, approximate score), loaded by the caller ahead of time
__device__ __forceinline__ void rank_resolve(const RankArgs& a, double last_cs, int64_t last_id, double eps, int q,
                                             int n, bool k32, int thr_mode, double kth, int cnt, int* ocnt,
                                             int* ores, int count_empty, int* oredo) {
  const int k = a.k;
  ocnt[q] = cnt;
  const bool full = last_id >= 0;
  // an empty last slot with score +inf: the scan's list may be incomplete (k_pool_select)
  const bool trunc = !full && last_cs == __builtin_huge_val();
  int res = trunc ? 0 : 1;
  if (full) {
    const double bound = last_cs + eps;
    if (n >= k) res = k32 ? (float)bound < (float)kth : bound < kth;
    else if (thr_mode == 0) res = 0;
    else res = thr_mode == 1 ? (bound < thr_low(a.thr)) : (bound <= thr_low(a.thr));
  }
  ores[q] = res;
  if (oredo && (res == 0 || (count_empty && cnt == 0))) atomicAdd(oredo, 1);
}

// Ranking pass (one 256-thread workgroup per query): the list's exact scores from the workspace, the
// (score desc, id asc) bitonic sort in LDS, the outputs (records gathered by list position), the count
// and the completeness proof as refine_big_body.
// The progressive search's final ranking fused into the re-rank's sort (one list per query, no arg-max
// fallback: hq_refine_final_ws): the survivors r < count in level-0 order, ranked by (overall desc, r asc)
// — k_progressive_final_big's order — K outputs with their records; the level-0 records are not written.
struct FinalOut {
  int K;
  int64_t* id;
  double* det;
  int* count;
  int rounds;  // 1: K <= kFinalRounds outputs by arg-max rounds where cheaper than the sort (option final_rounds)
};


// (round 6: a register-resident form — two entries per thread, in-wave partners by lane shuffles, LDS only
// across waves, NT = n2 / 2 — measured slower, 97.5 -> 121 us at M = 1000 and 20.8 -> 28.2 us at M = 100:
// profiles/r06_ab_scan_occ.txt; not kept)
// CAP: list entries the workgroup holds (a power of two >= kp): kMaxTopKBig, or 128 for the M = 100 lists
// (4 KB of LDS per workgroup instead of 33: many queries per CU)
template <int NT, int CAP = kMaxTopKBig>
__global__ __launch_bounds__(NT) void k_rank_sort(RankArgs a, const double* __restrict__ cs, double eps,
                                                   double* __restrict__ os, int64_t* __restrict__ oid,
                                                   int* __restrict__ ocnt, int* __restrict__ ores, int count_empty,
                                                   int* __restrict__ oredo, double* __restrict__ odet,
                                                   int* __restrict__ onext, FinalOut fin) {
  if (onext && blockIdx.x == 0 && threadIdx.x == 0) *onext = 0;  // the next batch's redo counter
  __shared__ double se[CAP];
  __shared__ int64_t sid[CAP];
  __shared__ int pos[CAP];
  __shared__ int fpos[CAP];
  __shared__ double rv[2][NT / 64];
  __shared__ int ri[2][NT / 64];
  __shared__ int red[NT / 64];
  __shared__ double csl[CAP];  // window ranking: the list's approximate scores (-inf: empty slot)
  __shared__ unsigned long long vmask[CAP / 64];  // valid entries, 64 list positions per word
  __shared__ int vpre[CAP / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kp = a.kp, k = a.k, W = 1 + a.cs.nseg;
  const int n2 = pow2_at_least(kp);
  const bool k32 = (a.thr_mode & kThrKey32) != 0;
  const int thr_mode = a.thr_mode & (kThrKey32 - 1);
  for (int q = blockIdx.x; q < a.Q; q += gridDim.x) {
    const int64_t base = (int64_t)q * kp;
    // the proof's inputs (the list's last slot) requested with the workspace reads, not after the sort
    const double last_cs = tid == 0 ? cs[base + kp - 1] : 0.0;
    const int64_t last_id = tid == 0 ? a.cid[base + kp - 1] : -1;
    int nv = 0;
    auto load = [&](int x) {
      const int64_t i = x < kp ? a.ws_id[base + x] : -1;
      se[x] = x < kp ? a.ws_sc[base + x] : -__builtin_huge_val();
      sid[x] = i;
      pos[x] = x;
      return i >= 0 ? 1 : 0;
    };
    for (int x = tid; x < n2; x += NT) {
      nv += load(x);
      if (a.win && n2 <= (CAP / NT) * NT) {
        csl[x] = x < kp && a.cid[base + x] >= 0 ? cs[base + x] : -__builtin_huge_val();
        fpos[x] = -1;
      }
    }
    nv = wsum64i(nv);
    if (lane == 0) red[wave] = nv;
    __syncthreads();
    int n = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) n += red[w];
    // Window ranking.  The list arrives in approximate-score order (k_pool_sort: approximate score desc, id
    // asc) and |exact - approximate| < eps (the completeness proof's own premise), so a valid entry's rank in
    // the (exact key desc, id asc) order is the count of valid entries whose approximate score lies more than
    // 2 eps above its own, plus its exact comparisons with the entries inside that window; invalid entries
    // follow in list order.  The result is checked — every rank taken once and every adjacent pair of valid
    // entries in order, which holds for the sorted order alone — and the bitonic sort below runs instead when
    // the check fails or a window passes kRankWin entries (runs of near-equal scores), so the ranking is the
    // sort's whatever the input.  Replaces the sort's 10 x 11 / 2 barrier stages by a few LDS reads per entry.
    bool sorted = false;
    constexpr int WE = CAP / NT;  // list entries per thread
    if (a.win && n2 <= WE * NT) {
      constexpr int kRankWin = 32;
      for (int c = wave; c < n2 / 64; c += NT / 64) {
        const unsigned long long m = __ballot(sid[64 * c + lane] >= 0);
        if (lane == 0) vmask[c] = m;
      }
      __syncthreads();
      if (tid < n2 / 64) {  // valid entries before each 64-position word
        int p = 0;
        for (int c = 0; c < tid; ++c) p += __popcll(vmask[c]);
        vpre[tid] = p;
      }
      __syncthreads();
      auto before_n = [&](int x) {  // valid entries at list positions < x
        return vpre[x >> 6] + __popcll(vmask[x >> 6] & ((1ull << (x & 63)) - 1ull));
      };
      const double wd = 2.0 * eps;
      bool bad = false;
      int rk[WE];
      double ms[WE];
      int64_t mi[WE];
#pragma unroll
      for (int e = 0; e < WE; ++e) {
        rk[e] = -1;
        ms[e] = 0.0;
        mi[e] = -1;
      }
#pragma unroll
      for (int e = 0; e < WE; ++e) {
        const int x = tid + NT * e;
        if (x >= n2) continue;
        __builtin_amdgcn_sched_barrier(0);  // one entry's window at a time (fewer live registers)
        const int64_t ix = sid[x];
        ms[e] = se[x];
        mi[e] = ix;
        if (ix < 0) {
          rk[e] = n + (x - before_n(x));
          continue;
        }
        const double ci = csl[x], kx = key_of(ms[e], k32);
        auto ahead = [&](int j) {  // valid entry j ranks before x
          const int64_t ij = sid[j];
          if (ij < 0) return 0;
          const double kj = key_of(se[j], k32);
          return (kj > kx || (kj == kx && ij < ix)) ? 1 : 0;
        };
        int lo = x;
#pragma unroll 1
        while (lo > 0 && csl[lo - 1] <= ci + wd && x - lo < kRankWin) --lo;
        if (lo > 0 && csl[lo - 1] <= ci + wd) bad = true;
        int r = before_n(lo);
#pragma unroll 1
        for (int j = lo; j < x; ++j) r += ahead(j);
        int hi = x + 1;
#pragma unroll 1
        while (hi < n2 && csl[hi] >= ci - wd && hi - x <= kRankWin) r += ahead(hi++);
        if (hi < n2 && csl[hi] >= ci - wd) bad = true;
        rk[e] = r;
      }
      bad = __syncthreads_or(bad);
      if (!bad) {
#pragma unroll
        for (int e = 0; e < WE; ++e) {
          const int r = rk[e];
          if (r >= 0 && r < n2) {
            se[r] = ms[e];
            sid[r] = mi[e];
            pos[r] = tid + NT * e;
            fpos[r] = tid + NT * e;
          }
        }
        __syncthreads();
        for (int r = tid; r < n2; r += NT) {
          if (fpos[r] < 0) bad = true;
          if (r + 1 < n) {
            const double k0 = key_of(se[r], k32), k1 = key_of(se[r + 1], k32);
            if (!(k0 > k1 || (k0 == k1 && sid[r] < sid[r + 1]))) bad = true;
          }
        }
        bad = __syncthreads_or(bad);
        if (bad) {  // the scattered arrays are not the sorted order: back to the list order for the sort
          for (int x = tid; x < n2; x += NT) load(x);
          __syncthreads();
        }
      }
      sorted = !bad;
    }
    if (!sorted)
    lds_bitonic(n2,
                [&](int x, int y) {
                  const int64_t ix = sid[x], iy = sid[y];
                  if (iy < 0) return ix >= 0;
                  const double kx = key_of(se[x], k32), ky = key_of(se[y], k32);
                  return ix >= 0 && (kx > ky || (kx == ky && ix < iy));
                },
                [&](int x, int y) {
                  const double te = se[x];
                  se[x] = se[y];
                  se[y] = te;
                  const int64_t ti = sid[x];
                  sid[x] = sid[y];
                  sid[y] = ti;
                  const int tp = pos[x];
                  pos[x] = pos[y];
                  pos[y] = tp;
                });
    const int cnt = n < k ? n : k;
    if (os)  // (the fused final ranking may go without the level-0 lists: hq_refine_final_ws)
      for (int r = tid; r < k; r += NT) {
        os[(int64_t)q * k + r] = r < cnt ? se[r] : -__builtin_huge_val();
        oid[(int64_t)q * k + r] = r < cnt ? sid[r] : -1;
      }
    if (odet) {  // records gathered by list position, four loads in flight per thread before the stores
      const double* __restrict__ rec = a.ws_rec;
      const int tot = k * W;
      for (int t0 = tid; t0 < tot; t0 += 4 * NT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int t = t0 + NT * u, r = t / W, w = t - r * W;
          v[u] = t < tot && r < cnt ? rec[(base + pos[r]) * W + w] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (t0 + NT * u < tot) odet[(int64_t)q * tot + t0 + NT * u] = v[u];
      }
    }
    if (tid == 0)
      rank_resolve(a, last_cs, last_id, eps, q, n, k32, thr_mode, n >= k ? se[k - 1] : -__builtin_huge_val(), cnt,
                   ocnt, ores, count_empty, oredo);
    __syncthreads();
    if (fin.id) {
      // survivors' overall keys in level-0 order (se is free: the proof has read se[k - 1])
      const double* __restrict__ rec = a.ws_rec;
      const int m2 = pow2_at_least(cnt > 2 ? cnt : 2);
      for (int r = tid; r < m2; r += NT) {
        se[r] = r < cnt ? key_of(rec[(base + pos[r]) * W], k32) : -__builtin_huge_val();
        fpos[r] = r;
      }
      __syncthreads();
      const int outn = cnt < fin.K ? cnt : fin.K;
      int lg = 1;
      while ((1 << lg) < cnt) ++lg;
      auto first = [](double x, int ix, double y, int iy) { return ix >= 0 && (iy < 0 || x > y || (x == y && ix < iy)); };
      if (fin.rounds && fin.K <= kFinalRounds && 3 * outn < lg * (lg + 1) / 2) {
        // outn rounds of the workgroup's first (overall desc, position asc) among the entries not yet taken
        constexpr int E = CAP / NT;
        double v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = tid + NT * e < cnt ? se[tid + NT * e] : 0.0;
        int taken = 0;
        for (int r = 0; r < outn; ++r) {
          double bv = 0.0;
          int bi = -1;
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int i = tid + NT * e;
            if (i < cnt && !((taken >> e) & 1) && first(v[e], i, bv, bi)) {
              bv = v[e];
              bi = i;
            }
          }
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const double v2 = __shfl_xor(bv, o, 64);
            const int i2 = __shfl_xor(bi, o, 64);
            if (first(v2, i2, bv, bi)) {
              bv = v2;
              bi = i2;
            }
          }
          if (lane == 0) {
            rv[r & 1][wave] = bv;
            ri[r & 1][wave] = bi;
          }
          __syncthreads();  // (the other buffer is rewritten only after the next round's barrier)
          bv = rv[r & 1][0];
          bi = ri[r & 1][0];
#pragma unroll
          for (int w = 1; w < NT / 64; ++w)
            if (first(rv[r & 1][w], ri[r & 1][w], bv, bi)) {
              bv = rv[r & 1][w];
              bi = ri[r & 1][w];
            }
          if (bi >= 0 && bi % NT == tid) taken |= 1 << (bi / NT);
          if (tid == 0) fpos[r] = bi;
        }
      } else {
        lds_bitonic(m2, [&](int x, int y) { return se[x] > se[y] || (se[x] == se[y] && fpos[x] < fpos[y]); },
                    [&](int x, int y) {
                      const double t = se[x];
                      se[x] = se[y];
                      se[y] = t;
                      const int tp = fpos[x];
                      fpos[x] = fpos[y];
                      fpos[y] = tp;
                    });
      }
      __syncthreads();
      for (int t = tid; t < fin.K * W; t += NT) {
        const int r = t / W, w = t - r * W;
        double val = 0.0;
        if (r < outn) {
          const int lr = fpos[r];
          val = rec[(base + pos[lr]) * W + w];
          if (w == 0) fin.id[(int64_t)q * fin.K + r] = sid[lr];
        } else if (w == 0) {
          fin.id[(int64_t)q * fin.K + r] = -1;
        }
        fin.det[(int64_t)q * fin.K * W + t] = val;
      }
      if (tid == 0) fin.count[q] = outn;
      __syncthreads();
    }
  }
}

// Short lists (kp <= 64, the M = 20 headline's 28 entries): k_rank_pairs and k_rank_sort in one kernel, one
// workgroup of NG 8-lane groups per query (NG >= kp): the entries' scores, ids and records stay in LDS, the
// (score desc, id asc) order is a rank count (each entry compares itself with the others), the outputs and
// the proof as k_rank_sort.  Replaces k_refine_lds (one thread per entry walking its row: 20.6 us per
// 1000-query batch).
// (round 6: at 3 waves per SIMD — 142 VGPRs, none of the 8 spilled at the 128-VGPR cap of 4 — 2-5% slower at
// M = 20: profiles/r06_ab_count_kernel.txt, rank_occ rows; not kept)
template <int PPL, int NG, int LID = 0>
__global__ __launch_bounds__(8 * NG) __attribute__((amdgpu_waves_per_eu(4))) void k_rank_small(RankArgs a, const double* __restrict__ cs, double eps,
                                                        double* __restrict__ os, int64_t* __restrict__ oid,
                                                        int* __restrict__ ocnt, int* __restrict__ ores,
                                                        int count_empty, int* __restrict__ oredo,
                                                        double* __restrict__ odet, int* __restrict__ onext,
                                                        FinalOut fin) {
  if (onext && blockIdx.x == 0 && threadIdx.x == 0) *onext = 0;  // the next batch's redo counter
  extern __shared__ __attribute__((aligned(16))) double cm[];
  constexpr int NT = 8 * NG;
  const int tid = threadIdx.x, g = tid >> 3, j = tid & 7;
  const int kp = a.kp, k = a.k, W = 1 + a.cs.nseg;
  const bool k32 = (a.thr_mode & kThrKey32) != 0;
  const int thr_mode = a.thr_mode & (kThrKey32 - 1);
  const int QW = coop_qw(a.cs), RW = coop_rw(a.cs);
  double* rq = cm;
  double* rg = cm + QW + g * RW;
  double* se = cm + QW + NG * RW;  // [NG] scores, [NG] ids, [NG x W] records, [NG] positions by rank
  int64_t* sid = reinterpret_cast<int64_t*>(se + NG);
  double* srec = se + 2 * NG;
  int* pos = reinterpret_cast<int*>(srec + NG * W);
  int* fpos = pos + NG;  // final ranking: survivor position by final rank
  __shared__ int red[NG / 8];
  __shared__ double s_last_cs;
  __shared__ int64_t s_last_id;
  for (int q = blockIdx.x; q < a.Q; q += gridDim.x) {
    // the proof's inputs (the list's last slot) requested with the staging loads, not after the ranking, and
    // parked in LDS (registers are this kernel's limit)
    if (tid == 0) {
      s_last_cs = cs[(int64_t)q * kp + kp - 1];
      s_last_id = a.cid[(int64_t)q * kp + kp - 1];
    }
    const int64_t c = rank_stage<PPL>(a, rq, rg, q, g, tid, NT, j);
    __syncthreads();
    if (g < kp) {
      double e;
      int64_t id;
      rank_score_t<LID>(a, rq, rg, c, j, srec + g * W, e, id);
      if (j == 0) {
        se[g] = e;
        sid[g] = id;
      }
    }
    __syncthreads();
    // rank of entry t: the entries before it in (valid first, key desc, id asc, position asc) order
    int nv = 0;
    if (tid < kp) {
      const int64_t it = sid[tid];
      const double kt = key_of(se[tid], k32);
      int r = 0;
      for (int u = 0; u < kp; ++u) {
        const int64_t iu = sid[u];
        const double ku = key_of(se[u], k32);
        const bool before = it < 0 ? (iu >= 0 || u < tid) : (iu >= 0 && (ku > kt || (ku == kt && iu < it)));
        r += before ? 1 : 0;
      }
      pos[r] = tid;
      nv = it >= 0 ? 1 : 0;
    }
    nv = wsum64i(nv);
    if ((tid & 63) == 0) red[tid >> 6] = nv;
    __syncthreads();
    int n = 0;
#pragma unroll
    for (int w = 0; w < NG / 8; ++w) n += red[w];
    const int cnt = n < k ? n : k;
    if (os)  // (the fused final ranking may go without the level-0 lists: hq_refine_final_ws)
      for (int r = tid; r < k; r += NT) {
        os[(int64_t)q * k + r] = r < cnt ? se[pos[r]] : -__builtin_huge_val();
        oid[(int64_t)q * k + r] = r < cnt ? sid[pos[r]] : -1;
      }
    if (odet)
      for (int t = tid; t < k * W; t += NT) {
        const int r = t / W, w = t - r * W;
        odet[(int64_t)q * k * W + t] = r < cnt ? srec[pos[r] * W + w] : 0.0;
      }
    if (tid == 0)
      rank_resolve(a, s_last_cs, s_last_id, eps, q, n, k32, thr_mode, n >= k ? se[pos[k - 1]] : -__builtin_huge_val(), cnt, ocnt,
                   ores, count_empty, oredo);
    if (fin.id) {
      // fused final ranking (k_progressive_final's order: overall desc, level-0 position asc) by rank counting
      const int outn = cnt < fin.K ? cnt : fin.K;
      if (tid < cnt) {
        const double ot = key_of(srec[pos[tid] * W], k32);
        int r = 0;
        for (int u = 0; u < cnt; ++u) {
          const double ou = key_of(srec[pos[u] * W], k32);
          r += (ou > ot || (ou == ot && u < tid)) ? 1 : 0;
        }
        if (r < fin.K) fpos[r] = tid;
      }
      __syncthreads();
      for (int t = tid; t < fin.K * W; t += NT) {
        const int r = t / W, w = t - r * W;
        double val = 0.0;
        if (r < outn) {
          const int e = pos[fpos[r]];
          val = srec[e * W + w];
          if (w == 0) fin.id[(int64_t)q * fin.K + r] = sid[e];
        } else if (w == 0) {
          fin.id[(int64_t)q * fin.K + r] = -1;
        }
        fin.det[(int64_t)q * fin.K * W + t] = val;
      }
      if (tid == 0) fin.count[q] = outn;
    }
    __syncthreads();
  }
}

// shapes of the cooperative re-rank: every segment <= 128 values, L even, record width <= kCoopMaxW,
// <= 10 16-byte row pieces per lane; 0 = not supported
static int coop_ppl(const SegInfo& si) {
  if (!seg_small(si) || si.L % 2 != 0 || 1 + si.nseg > kCoopMaxW) return 0;
  const int ppl = (si.L / 2 + 2 * si.nseg + 7) / 8;
  return ppl <= 6 ? 6 : (ppl <= 10 ? 10 : 0);
}

static size_t refine_ws_bytes(int Q, int kp, int L) {
  if (Q <= 0 || kp <= 0 || L <= 0) return 0;
  SegInfo si;
  seg_info(L, si);
  return (size_t)Q * kp * (16 + 8 * (size_t)(1 + si.nseg)) + 256;
}

// k_progressive_final for M > 64: the survivors (one list: its valid prefix, counted by the whole
// workgroup; R lists: wave 0 merges them, final_survivors) ordered by (overall desc, survivor position asc)
// — the reference's stable sort.  Only the first K are needed: K <= kFinalRounds takes them by K rounds of a
// workgroup arg-max over register-held overall scores (one barrier per round); larger K sorts them whole
// (bitonic in LDS).  Round 4's form sorted all n (1024 keys at M = 1000, 55 bitonic stages) for K = 10 and
// read the single list's validity from one wave.
__global__ __launch_bounds__(256) void k_progressive_final_big(int R, int Q, int M, int W,
                                                               const double* __restrict__ s0,
                                                               const int64_t* __restrict__ ids,
                                                               const double* __restrict__ det,
                                                               const double* __restrict__ best,
                                                               const int64_t* __restrict__ best_id,
                                                               const double* __restrict__ best_det, int K,
                                                               int64_t* __restrict__ out_id,
                                                               double* __restrict__ out_det,
                                                               int* __restrict__ out_count, int flags) {
  __shared__ int sel[kMaxTopKBig];
  __shared__ double ovs[kMaxTopKBig];
  __shared__ int pos[kMaxTopKBig];
  __shared__ double rv[2][4];
  __shared__ int ri[2][4];
  __shared__ int red[4];
  __shared__ int sn;
  __shared__ int64_t sfb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool k32 = (flags & 1) != 0;
  auto first = [](double a, int ia, double b, int ib) { return ia >= 0 && (ib < 0 || a > b || (a == b && ia < ib)); };
  for (int q = blockIdx.x; q < Q; q += gridDim.x) {
    if (R == 1) {  // one list in (score desc, id asc) order, its valid entries first
      int c = 0;
      for (int i = tid; i < M; i += 256) {
        const bool v = ids[(int64_t)q * M + i] >= 0;
        c += v ? 1 : 0;
        sel[i] = i;
      }
      c = wsum64i(c);
      if (lane == 0) red[wave] = c;
      __syncthreads();
      if (tid == 0) {
        int n = red[0] + red[1] + red[2] + red[3];
        int64_t fb = -1;
        if (n == 0 && best_id[q] >= 0) {  // none passed the threshold: the first arg-max (:295-298)
          n = 1;
          fb = best_id[q];
        }
        sn = n;
        sfb = fb;
      }
    } else if (tid < 64) {
      int64_t fb;
      const int n = final_survivors(R, Q, M, q, s0, ids, best, best_id, sel, &fb, k32);
      if (tid == 0) {
        sn = n;
        sfb = fb;
      }
    }
    __syncthreads();
    const int n = sn;
    const int64_t fb_id = sfb;
    const double* rowbase = fb_id >= 0 ? best_det : det;
    auto row_of = [&](int v) -> int64_t {
      const int64_t rq = (int64_t)(v >> 16) * Q + q;
      return fb_id >= 0 ? rq : rq * M + (v & 0xFFFF);
    };
    const int outn = n < K ? n : K;
    // rounds (a wave reduction each, ~3 bitonic stages of work) when cheaper than the whole sort
    int lg = 1;
    while ((1 << lg) < n) ++lg;
    if (!(flags & 2) && K <= kFinalRounds && 3 * outn < lg * (lg + 1) / 2) {
      // K rounds of the workgroup's first (overall desc, position asc) among the entries not yet taken
      double v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = tid + 256 * e;
        v[e] = i < n ? key_of(rowbase[row_of(sel[i]) * W], k32) : 0.0;
      }
      int taken = 0;
      for (int r = 0; r < outn; ++r) {
        double bv = 0.0;
        int bi = -1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = tid + 256 * e;
          if (i < n && !((taken >> e) & 1) && first(v[e], i, bv, bi)) {
            bv = v[e];
            bi = i;
          }
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const double v2 = __shfl_xor(bv, o, 64);
          const int i2 = __shfl_xor(bi, o, 64);
          if (first(v2, i2, bv, bi)) {
            bv = v2;
            bi = i2;
          }
        }
        if (lane == 0) {
          rv[r & 1][wave] = bv;
          ri[r & 1][wave] = bi;
        }
        __syncthreads();  // (the other buffer is rewritten only after the next round's barrier)
        bv = rv[r & 1][0];
        bi = ri[r & 1][0];
#pragma unroll
        for (int w = 1; w < 4; ++w)
          if (first(rv[r & 1][w], ri[r & 1][w], bv, bi)) {
            bv = rv[r & 1][w];
            bi = ri[r & 1][w];
          }
        if ((bi & 255) == tid) taken |= 1 << (bi >> 8);
        if (tid == 0) pos[r] = bi;
      }
    } else {
      const int n2 = pow2_at_least(n);
      for (int i = tid; i < n2; i += 256) {
        ovs[i] = i < n ? key_of(rowbase[row_of(sel[i]) * W], k32) : -__builtin_huge_val();
        pos[i] = i;
      }
      __syncthreads();
      lds_bitonic(n2, [&](int a, int b) { return ovs[a] > ovs[b] || (ovs[a] == ovs[b] && pos[a] < pos[b]); },
                  [&](int a, int b) {
                    const double to = ovs[a];
                    ovs[a] = ovs[b];
                    ovs[b] = to;
                    const int tp = pos[a];
                    pos[a] = pos[b];
                    pos[b] = tp;
                  });
    }
    __syncthreads();
    for (int t = tid; t < K * W; t += 256) {  // one record value per thread
      const int r = t / W, w = t - r * W;
      double val = 0.0;
      if (r < outn) {
        const int64_t oi = row_of(sel[pos[r]]);
        val = rowbase[oi * W + w];
        if (w == 0) out_id[(int64_t)q * K + r] = fb_id >= 0 ? fb_id : ids[oi];
      } else if (w == 0) {
        out_id[(int64_t)q * K + r] = -1;
      }
      out_det[(int64_t)q * K * W + t] = val;
    }
    if (tid == 0) out_count[q] = outn;
    __syncthreads();
  }
}

// S7: (cos + 1) / 2, 0 if a norm is 0 (rag/search/engine.py:622-660, 1025-1051)
__global__ __launch_bounds__(256) void k_cosine(const float* __restrict__ A, int Q, const float* __restrict__ B,
                                                int64_t N, int K, double* __restrict__ out) {
  const int64_t total = (int64_t)Q * N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(t / N);
    const int64_t c = t % N;
    const float* a = A + (int64_t)q * K;
    const float* b = B + c * K;
    double dot = 0.0, na = 0.0, nb = 0.0;
    for (int i = 0; i < K; ++i) {
      const double x = a[i], y = b[i];
      dot = fma(x, y, dot);
      na = fma(x, x, na);
      nb = fma(y, y, nb);
    }
    double r = 0.0;
    if (na != 0.0 && nb != 0.0) r = (dot / (sqrt(na) * sqrt(nb)) + 1.0) / 2.0;
    out[t] = r;
  }
}

static int rs_for(int kp) {
  int r = kp < 2 ? 2 : kp;
  while ((r % 32) != 2) ++r;
  return r;
}

static size_t scan_lds_bytes(int rs, int nsu, int K) {
  return (size_t)8 * (kCB * rs + kCB * nsu * 4 + kQB * nsu * 4 + 4 * 16 * kCB + kQB * K) + (size_t)8 * kQB * K +
         (size_t)8 * kQB + (size_t)8 * kQB + (size_t)4 * kQB + 64;
}

static void scan_geometry(int Q, int64_t N, int& nqb, int& nchunks, int64_t& chunk_len) {
  nqb = (Q + kQB - 1) / kQB;
  // aim for ~2 waves of workgroups over 256 CUs; nchunks multiple of 8 (XCD mapping), <= 512
  int64_t target = (2048 + nqb - 1) / nqb;
  if (target < 8) target = 8;
  int64_t max_chunks = (N + kCB - 1) / kCB;
  if (target > max_chunks) target = max_chunks;
  if (target > 512) target = 512;
  nchunks = (int)(((target + 7) / 8) * 8);
  if (nchunks < 8) nchunks = 8;
  chunk_len = (N + nchunks - 1) / nchunks;
  chunk_len = ((chunk_len + kCB - 1) / kCB) * kCB;
  if (chunk_len < kCB) chunk_len = kCB;
}

// k_scan0: ~16 resident waves per CU-pair of rounds; nchunks multiple of 8 (XCD mapping), <= 512
static void scan0_geometry(int Q, int64_t N, int& nqb, int& nchunks, int64_t& chunk_len, int qw = kQW, int occ = 4) {
  nqb = (Q + qw - 1) / qw;
  // ~4096 waves of 64 queries (4 per SIMD); 128-query waves (k_scan0g<.., 8>, 3 per SIMD): one round of 3072;
  // occ 3 (option scan_occ 3: 64-query waves at 3 per SIMD, deeper prefetch): one round of 3072
  const int64_t waves = qw <= kQW ? (occ == 3 ? 3072LL : 4096LL * (kQW / qw)) : 3072;
  int64_t target = (waves + nqb - 1) / nqb;
  int64_t max_chunks = (N + kCS - 1) / kCS;
  if (target > max_chunks) target = max_chunks;
  if (target > 512) target = 512;
  nchunks = (int)(((target + 7) / 8) * 8);
  if (nchunks < 8) nchunks = 8;
  chunk_len = (N + nchunks - 1) / nchunks;
  chunk_len = ((chunk_len + kCS - 1) / kCS) * kCS;
  if (chunk_len < kCS) chunk_len = kCS;
}

// top-T sample pass (k_sample_topf): same stride rule as the histogram pass; ~2048 waves (no per-wave
// setup cost, so more waves only add occupancy), chunks a multiple of 8 (XCD map) and of kCS rows
static void sample_top_geometry(int Q, int64_t N, int64_t& stride, int64_t& S, int& nqb, int& nchunks,
                                int64_t& chunk_len) {
  const int64_t sd = opt(OPT_SAMPLE_STRIDE, 16) > 0 ? opt(OPT_SAMPLE_STRIDE, 16) : 16;  // A/B option
  stride = N >= sd * 4096 ? sd : (N / 4096 > 1 ? N / 4096 : 1);
  S = sample_rows_tiled(N, stride);  // whole 16-row tiles (k_sample_topf)
  nqb = (Q + kQW - 1) / kQW;
  const int waves = opt(OPT_SAMPLE_WAVES, 2048) > 0 ? (int)opt(OPT_SAMPLE_WAVES, 2048) : 2048;
  int64_t target = (waves + nqb - 1) / nqb;
  const int64_t max_chunks = (S + kCS - 1) / kCS;
  if (target > max_chunks) target = max_chunks;
  if (target > 64 * kKthReg / (4 * kTopT)) target = 64 * kKthReg / (4 * kTopT);  // k_sample_kth pool in registers
  nchunks = (int)(((target + 7) / 8) * 8);
  if (nchunks < 8) nchunks = 8;
  chunk_len = (S + nchunks - 1) / nchunks;
  chunk_len = ((chunk_len + kCS - 1) / kCS) * kCS;
}
static size_t sample_top_bytes(int Q, int64_t N) {
  int64_t stride, S, chunk_len;
  int nqb, nchunks;
  sample_top_geometry(Q, N, stride, S, nqb, nchunks, chunk_len);
  return (size_t)Q * 4 * nchunks * kTopT * 4;
}

// K' of the sampled starting threshold (a stride-s sample): the smallest K' with P(Binomial(k, 1/s) >= K')
// <= 1e-7, the chance that the sample holds K' of the corpus's k best pairs — only then can a pool end with
// fewer than k entries although more pass the caller's threshold (k_pool_select marks such a pool and the
// dense exact path answers the query).  k = 28 (the M = 20 headline): 12; k = 108: 24; k = 1008: 107.
static int sample_kprime(int k, int64_t stride) {
  if (stride <= 1 || k <= 1) return k;
  const double p = 1.0 / (double)stride, lp = log(p), lq = log1p(-p), lk = lgamma((double)k + 1.0);
  double tail = 0.0;
  for (int i = k; i >= 1; --i) {
    tail += exp(lk - lgamma((double)i + 1.0) - lgamma((double)(k - i) + 1.0) + i * lp + (k - i) * lq);
    if (tail > 1e-7) return i + 1 <= k ? i + 1 : k;
  }
  return 1;
}

// K' actually used: option sample_kth (0 = k, a provable bound) or the rule above; dense samples (stride
// below 16, small corpora) always k
static int scan_kprime(int k, int64_t stride) {
  int kp = (int)opt(OPT_SAMPLE_KTH, -1);
  if (kp < 0) kp = sample_kprime(k, stride);
  if (kp <= 0 || kp > k || stride < 16) kp = k;
  return kp;
}

// per-query pool capacity: k <= 64 keeps nchunks x k entries (a pool then never overflows); a long list
// (k > 64) is sized from the sample: ~stride x K' entries pass its starting threshold, capacity 3x that plus
// 1024 as a power of two, at most the corpus (an overflowing pool marks its query for the dense path)
static int pool_cap_for(int nchunks, int k, int64_t N, int64_t stride, int kprime) {
  if (k <= kMaxTopK) return nchunks * k;
  const int64_t want = 3 * stride * (int64_t)kprime + 1024;
  int64_t c = 4096;
  while (c < want && c < (int64_t(1) << 22)) c <<= 1;
  const int64_t n64 = (N + 63) / 64 * 64;
  return (int)(c < n64 ? c : n64);
}

static size_t scan0_lists_bytes(int Q, int64_t N, int k, int nchunks) {
  if (k <= kMaxTopK) return (size_t)nchunks * Q * k * 16;
  int64_t stride, S, chunk_len;
  int nqb, sn;
  sample_top_geometry(Q, N, stride, S, nqb, sn, chunk_len);
  const size_t b = (size_t)Q * pool_cap_for(nchunks, k, N, stride, scan_kprime(k, stride)) * 8;
  return (b + 255) & ~(size_t)255;
}

static size_t scan0_ws_bytes(int Q, int64_t N, int k) {
  int nqb, nchunks, nqb2, nchunks2;
  int64_t chunk_len, chunk_len2;
  scan0_geometry(Q, N, nqb, nchunks, chunk_len);
  scan0_geometry(Q, N, nqb2, nchunks2, chunk_len2, 32);
  if (nchunks2 > nchunks) nchunks = nchunks2;
  if (opt(OPT_SCAN_NB, 4) == 8) {  // the 128-query scan's geometry (A/B option) only when selected
    scan0_geometry(Q, N, nqb2, nchunks2, chunk_len2, 128);
    if (nchunks2 > nchunks) nchunks = nchunks2;
  }
  // lists / pools + global thresholds + sample histogram + starting thresholds + pool counts + sample tops
  return scan0_lists_bytes(Q, N, k, nchunks) + (size_t)Q * 8 + (size_t)Q * kBins * 4 + (size_t)Q * 8 + (size_t)Q * 4 +
         sample_top_bytes(Q, N) + (size_t)Q * sizeof(QConst) + (size_t)N * 4 + 1024;
}

#ifdef HQ_DIAG
// sample pass: stride 16 once the corpus is large, else a sample of ~4096 rows (the whole corpus
// below that); chunks of <= 65520 rows (u16 histogram counters), ~1024 waves (a wave has a fixed
// cost: histogram init and flush)
static void sample_geometry(int Q, int64_t N, int64_t& stride, int64_t& S, int& nqb, int& nchunks,
                            int64_t& chunk_len, bool tiled) {
  const int64_t sd = opt(OPT_SAMPLE_STRIDE, 16) > 0 ? opt(OPT_SAMPLE_STRIDE, 16) : 16;  // A/B option
  stride = N >= sd * 4096 ? sd : (N / 4096 > 1 ? N / 4096 : 1);
  S = tiled ? sample_rows_tiled(N, stride) : (N + stride - 1) / stride;  // f32 (split) samples: whole tiles
  nqb = (Q + kQW - 1) / kQW;
  const int waves = opt(OPT_SAMPLE_WAVES, 1024) > 0 ? (int)opt(OPT_SAMPLE_WAVES, 1024) : 1024;
  int64_t target = (waves + nqb - 1) / nqb;
  const int64_t max_chunks = (S + kCS - 1) / kCS;
  if (target > max_chunks) target = max_chunks;
  if (target < (S + 65519) / 65520) target = (S + 65519) / 65520;
  nchunks = (int)(((target + 7) / 8) * 8);
  chunk_len = (S + nchunks - 1) / nchunks;
  chunk_len = ((chunk_len + kCS - 1) / kCS) * kCS;
}
#endif  // HQ_DIAG

static int launch_scan0f(const Scan0Args& a, hipStream_t s) {
  const size_t lds = (size_t)kQW * a.K * 8;
  HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_scan0f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_scan0f, dim3(a.nqb * a.nchunks), dim3(64), lds, s, a);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

#ifdef HQ_DIAG
template <int KS, bool F32>
static int launch_sample(const SampleArgs& a, hipStream_t s) {
  const size_t lds = (size_t)kQW * kHRow * 4;
  const void* fn = F32 ? (const void*)k_sample_histf : (const void*)k_sample_hist<KS>;
  HQ_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if constexpr (F32) hipLaunchKernelGGL(k_sample_histf, dim3(a.nqb * a.nchunks), dim3(64), lds, s, a);
  else hipLaunchKernelGGL((k_sample_hist<KS>), dim3(a.nqb * a.nchunks), dim3(64), lds, s, a);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int KS, bool F32>
static int launch_scan0(const Scan0Args& a, hipStream_t s) {
  if constexpr (F32) return launch_scan0f(a, s);
  const size_t lds = (size_t)kQW * 32 + (size_t)kQW * a.K * 12;
  HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_scan0<KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_scan0<KS>), dim3(a.nqb * a.nchunks), dim3(64), lds, s, a);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <bool F32>
static int scan0_dispatch(int ks, const Scan0Args& b, const SampleArgs* sa, hipStream_t s) {
  int rc;
  if (sa) {
    switch (ks) {
      case 1: rc = launch_sample<1, F32>(*sa, s); break;
      case 2: rc = launch_sample<2, F32>(*sa, s); break;
      case 3: rc = launch_sample<3, F32>(*sa, s); break;
      case 4: rc = launch_sample<4, F32>(*sa, s); break;
      case 5: rc = launch_sample<5, F32>(*sa, s); break;
      case 6: rc = launch_sample<6, F32>(*sa, s); break;
      case 7: rc = launch_sample<7, F32>(*sa, s); break;
      default: rc = launch_sample<8, F32>(*sa, s); break;
    }
    return rc;
  }
  switch (ks) {
    case 1: rc = launch_scan0<1, F32>(b, s); break;
    case 2: rc = launch_scan0<2, F32>(b, s); break;
    case 3: rc = launch_scan0<3, F32>(b, s); break;
    case 4: rc = launch_scan0<4, F32>(b, s); break;
    case 5: rc = launch_scan0<5, F32>(b, s); break;
    case 6: rc = launch_scan0<6, F32>(b, s); break;
    case 7: rc = launch_scan0<7, F32>(b, s); break;
    default: rc = launch_scan0<8, F32>(b, s); break;
  }
  return rc;
}

#endif  // HQ_DIAG

// level-0 scan: top-T sample pass -> starting thresholds -> k_scan0f -> k_pool_select (split-f16
// contraction, f32 == true).  DIAG builds keep the superseded forms for A/B: the f64 wave-level scan
// k_scan0 (f32 == false, merged by k_merge) and the histogram sample pass (option sample_hist).
static int scan0_run(bool f32, int ks, const double* Zq, const double* Sq, const _Float16* Zq16, const float* Sq32,
                     int Q, const double* Zc, const double* Sc, const _Float16* Zc16, const float* Sc32, int64_t N,
                     const SegInfo& si, int k, double threshold, int thr_mode, int64_t id_base, void* workspace,
                     double* out_score, int64_t* out_id, hipStream_t s, const int* corpus_flags = nullptr) {
#ifndef HQ_DIAG
  if (!f32) return fail(HQ_E_UNSUPPORTED, "the f64 level-0 scan exists only in DIAG builds");
#endif
  Scan0Args b;
  b.Zq = Zq; b.Sq = Sq; b.Q = Q; b.Zc = Zc; b.Sc = Sc; b.N = N;
  b.Zq32 = nullptr; b.Zc32 = nullptr; b.Zq16 = Zq16; b.Zc16 = Zc16; b.Sq32 = Sq32; b.Sc32 = Sc32;
  b.Lp = si.Lp; b.nseg = si.nseg; b.P0 = si.plen[0];
  b.inv_m = si.inv_m[0];
  b.c1 = 0.35 * si.inv_m[0];
  b.K = k;
  b.thr0 = thr_mode == 0 ? -__builtin_huge_val() : threshold;
  b.id_base = id_base;
  b.expt = 0;
  b.dbg = nullptr;
#ifdef HQ_DIAG
  b.expt = (int)opt(OPT_SCAN_EXPT, 0);
  static unsigned long long* dbg = nullptr;
  if (b.expt == 3) {
    if (!dbg) HQ_CHECK_HIP(hipMalloc(&dbg, 64));
    HQ_CHECK_HIP(hipMemsetAsync(dbg, 0, 64, s));
  }
  b.dbg = dbg;
#endif
  // option scan_nb 8: 128-query waves (k_scan0g<1, PF, 8>) and their geometry
  const int scan_nb = f32 && opt(OPT_SCAN_NB, 4) == 8 && opt(OPT_SCAN_WPB, 1) != 4 ? 8 : 4;
  // 3 waves per SIMD (default since round 6; 168 VGPRs: room for a 6-step prefetch), 3072 waves: the list-1008
  // scan 197 -> 161 us (profiles/r06_ab_scan_occ.txt).  Option scan_occ 4: the round-5 form (4 per SIMD, 4 steps)
  const int socc = f32 && scan_nb == 4 && opt(OPT_SCAN_WPB, 1) != 4 && opt(OPT_SCAN_OCC, 3) == 3 ? 3 : 4;
  scan0_geometry(Q, N, b.nqb, b.nchunks, b.chunk_len, 16 * scan_nb, socc);
  uint8_t* ws = reinterpret_cast<uint8_t*>(workspace);
  b.ws_score = reinterpret_cast<double*>(ws);
  b.ws_id = reinterpret_cast<int64_t*>(ws + (size_t)b.nchunks * Q * k * 8);
  // [lists / pools][gtau Q x 8][hist Q x kBins x 4][pool_n Q x 4][th0 Q x 8][sample tops]: the zeroed
  // regions are adjacent, so one memset clears them
  const size_t lists = scan0_lists_bytes(Q, N, k, b.nchunks);
  b.gtau = reinterpret_cast<unsigned long long*>(ws + lists);
  unsigned int* hist = reinterpret_cast<unsigned int*>(ws + lists + (size_t)Q * 8);
  b.pool_n = reinterpret_cast<int*>(ws + lists + (size_t)Q * 8 + (size_t)Q * kBins * 4);
  double* th0 = reinterpret_cast<double*>(ws + lists + (size_t)Q * 8 + (size_t)Q * kBins * 4 + (size_t)Q * 4);
  b.th0 = nullptr;
  // f32 path: per-query pools in the list area (pool_cap_for: nchunks * k entries for k <= 64)
  int64_t s_stride, s_S, s_len;
  int s_nqb, s_nch;
  sample_top_geometry(Q, N, s_stride, s_S, s_nqb, s_nch, s_len);
  b.pool_cap = pool_cap_for(b.nchunks, k, N, s_stride, scan_kprime(k, s_stride));
  b.pool_s = reinterpret_cast<float*>(ws);
  b.pool_i = reinterpret_cast<int*>(ws + (size_t)Q * b.pool_cap * 4);
  // option scan_nosample: no sample pass, the scan starts from the caller's threshold
  const bool sample = !opt_on(OPT_SCAN_NOSAMPLE);
  bool top_sample = sample && f32;
#ifdef HQ_DIAG
  if (top_sample && opt(OPT_SCAN_VARIANT, 0) == 100) top_sample = false;  // the histogram sample pass
#endif
  // K' of the starting threshold: the sample's K'-th best (statistical for K' < k: pools left short are
  // marked for the exact path, k_pool_select); option sample_kth = 0 -> k (a provable bound)
  int sample_kth = scan_kprime(k, s_stride);
  float* top = reinterpret_cast<float*>(ws + lists + (size_t)Q * 8 + (size_t)Q * kBins * 4 + (size_t)Q * 4 +
                                        (size_t)Q * 8);
  // k_scan0g (default; option scan_variant 1 = the list-based k_scan0f): per-query constants after the
  // sample tops, 256-B aligned
  // (the list kernel keeps one list entry per lane and nchunks x k pool slots: k <= 64 only, so longer
  // lists always take the queue scan whatever the option says)
  const bool queue_scan = f32 && (opt(OPT_SCAN_VARIANT, 0) != 1 || k > kMaxTopK);
  const size_t qc_off = ((size_t)(reinterpret_cast<uint8_t*>(top) - ws) + sample_top_bytes(Q, N) + 255) & ~(size_t)255;
  QConst* qc = queue_scan ? reinterpret_cast<QConst*>(ws + qc_off) : nullptr;
  b.qconst = qc;
  int* flag_n = reinterpret_cast<int*>(ws + ((qc_off + (size_t)Q * sizeof(QConst) + 255) & ~(size_t)255));
  int* flag_list = flag_n + 64;
  // (the top-T sample has no histogram and k_sample_kth clears gtau and pool_n per query)
  if (!top_sample)
    HQ_CHECK_HIP(hipMemsetAsync(b.gtau, 0, (size_t)Q * 8 + (sample ? (size_t)Q * kBins * 4 : 0) + (f32 ? (size_t)Q * 4 : 0),
                                s));
  if (f32 && !sample) HQ_CHECK_HIP(hipMemsetAsync(b.pool_n, 0, sizeof(int) * Q, s));
  int rc;
  if (top_sample) {
    SampleArgs sa;
    sa.Zq = Zq; sa.Sq = Sq; sa.Q = Q; sa.Zc = Zc; sa.Sc = Sc; sa.N = N;
    sa.Zq32 = nullptr; sa.Zc32 = nullptr; sa.Zq16 = Zq16; sa.Zc16 = Zc16; sa.Sq32 = Sq32; sa.Sc32 = Sc32;
    sa.Lp = b.Lp; sa.nseg = b.nseg; sa.P0 = b.P0; sa.inv_m = b.inv_m; sa.c1 = b.c1;
    sample_top_geometry(Q, N, sa.stride, sa.S, sa.nqb, sa.nchunks, sa.chunk_len);
    sa.hist = nullptr;
    sa.top = top;
    sa.K = k;
    // option sample_variant 1: the full-filter sample pass (k_sample_topf)
    if (opt(OPT_SAMPLE_VARIANT, 0) == 1)
      hipLaunchKernelGGL(k_sample_topf, dim3(sa.nqb * sa.nchunks), dim3(64), 0, s, sa);
    else if (opt(OPT_SAMPLE_HI, 0) == 1)  // hi.hi step loop + split G epilogue: 58 vs 34 us (the epilogue's loads)
      hipLaunchKernelGGL(k_sample_topg<true>, dim3(sa.nqb * sa.nchunks), dim3(64), 0, s, sa);
    else
      hipLaunchKernelGGL(k_sample_topg<false>, dim3(sa.nqb * sa.nchunks), dim3(64), 0, s, sa);
    HQ_CHECK_LAUNCH();
    const int mg = Q < 8192 ? Q : 8192;
    launch_kth(mg, s, (const float*)top, 4 * sa.nchunks, Q, sample_kth, (double)kMarginF, th0, b.gtau, b.pool_n, Sq32,
               b.thr0, b.inv_m, qc);
    HQ_CHECK_LAUNCH();
    b.th0 = th0;
  }
#ifdef HQ_DIAG
  else if (sample) {
    SampleArgs sa;
    sa.top = nullptr;
    sa.Zq = Zq; sa.Sq = Sq; sa.Q = Q; sa.Zc = Zc; sa.Sc = Sc; sa.N = N;
    sa.Zq32 = nullptr; sa.Zc32 = nullptr; sa.Zq16 = Zq16; sa.Zc16 = Zc16; sa.Sq32 = Sq32; sa.Sc32 = Sc32;
    sa.Lp = b.Lp; sa.nseg = b.nseg; sa.P0 = b.P0; sa.inv_m = b.inv_m; sa.c1 = b.c1;
    sample_geometry(Q, N, sa.stride, sa.S, sa.nqb, sa.nchunks, sa.chunk_len, f32);
    sa.hist = hist;
    sa.K = k;
    rc = f32 ? scan0_dispatch<true>(ks, b, &sa, s) : scan0_dispatch<false>(ks, b, &sa, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_hist_tau, dim3((Q + 255) / 256), dim3(256), 0, s, (const unsigned int*)hist, Q, k,
                       f32 ? (double)kMarginF : 1e-12, th0);
    HQ_CHECK_LAUNCH();
    b.th0 = th0;
  }
#else
  (void)hist;
  rc = HQ_OK;
#endif
  if (queue_scan) {
    if (!top_sample) {  // no sample pass: the constants from the caller's threshold (and pool counts cleared)
      hipLaunchKernelGGL(k_scan_qprep, dim3((Q + 255) / 256), dim3(256), 0, s, Sq32, Q, b.thr0, b.inv_m, qc, b.pool_n);
      HQ_CHECK_LAUNCH();
    }
    if (corpus_flags) {  // the corpus's flagged rows listed once (hq_seg_flag_rows): [count, rows...]
      flag_n = const_cast<int*>(corpus_flags);
      flag_list = flag_n + 1;
    } else {
      HQ_CHECK_HIP(hipMemsetAsync(flag_n, 0, sizeof(int), s));
      const int64_t fb = (N + 255) / 256;
      hipLaunchKernelGGL(k_flag_rows, dim3((unsigned)(fb < 4096 ? fb : 4096)), dim3(256), 0, s, Sc32, N, flag_list,
                         flag_n);
      HQ_CHECK_LAUNCH();
    }
    // options scan_wpb: waves per block (1 = one wave per block, each reading its own fragments);
    // scan_pf: prefetch distance in steps (2, 3, 4, 6, 8; 4 measured best at 4 waves per SIMD: 4.73M vs
    // 4.64M QPS at 2, 3.02M at 6 where the queue spills)
    const int pf = (int)opt(OPT_SCAN_PF, socc == 3 ? 6 : 4);
    if (opt(OPT_SCAN_WPB, 1) == 4) {
      const dim3 g4((b.nqb + 3) / 4 * b.nchunks);
      if (pf == 4) hipLaunchKernelGGL((k_scan0g<4, 4>), g4, dim3(256), 0, s, b);
      else if (pf == 3) hipLaunchKernelGGL((k_scan0g<4, 3>), g4, dim3(256), 0, s, b);
      else hipLaunchKernelGGL((k_scan0g<4, 2>), g4, dim3(256), 0, s, b);
    } else {
      const dim3 g1(b.nqb * b.nchunks);
      if (scan_nb == 8) hipLaunchKernelGGL((k_scan0g<1, 2, 8>), g1, dim3(64), 0, s, b);
      else if (opt_on(OPT_SCAN_SPLIT3)) hipLaunchKernelGGL((k_scan0g<1, 2, 4, false>), g1, dim3(64), 0, s, b);
      else if (opt(OPT_SCAN_OCC, 3) == 5) {
        if (pf == 4) hipLaunchKernelGGL((k_scan0g<1, 4, 4, true, 5>), g1, dim3(64), 0, s, b);
        else hipLaunchKernelGGL((k_scan0g<1, 2, 4, true, 5>), g1, dim3(64), 0, s, b);
      } else if (socc == 3) {
        if (pf == 8) hipLaunchKernelGGL((k_scan0g<1, 8, 4, true, 3>), g1, dim3(64), 0, s, b);
        else if (pf == 6) hipLaunchKernelGGL((k_scan0g<1, 6, 4, true, 3>), g1, dim3(64), 0, s, b);
        else hipLaunchKernelGGL((k_scan0g<1, 4, 4, true, 3>), g1, dim3(64), 0, s, b);
      } else {  // 4 waves per SIMD (measured best: 4.64M vs 1.41M QPS at 5 with the drain gate)
        if (pf == 8) hipLaunchKernelGGL((k_scan0g<1, 8, 4, true, 4>), g1, dim3(64), 0, s, b);
        else if (pf == 6) hipLaunchKernelGGL((k_scan0g<1, 6, 4, true, 4>), g1, dim3(64), 0, s, b);
        else if (pf == 4) hipLaunchKernelGGL((k_scan0g<1, 4, 4, true, 4>), g1, dim3(64), 0, s, b);
        else if (pf == 3) hipLaunchKernelGGL((k_scan0g<1, 3, 4, true, 4>), g1, dim3(64), 0, s, b);
        else hipLaunchKernelGGL((k_scan0g<1, 2, 4, true, 4>), g1, dim3(64), 0, s, b);
      }
    }
    HQ_CHECK_LAUNCH();
    // flagged rows are rare (usually none): scored inside k_pool_select, before it reads the pools
  } else {
#ifdef HQ_DIAG
    rc = f32 ? scan0_dispatch<true>(ks, b, nullptr, s) : scan0_dispatch<false>(ks, b, nullptr, s);
#else
    rc = launch_scan0f(b, s);
#endif
  }
  if (rc) return rc;
  if (f32) {
    launch_pool_select(k, s, Q, b.pool_s, b.pool_i, b.pool_n, b.pool_cap, id_base, out_score, out_id,
                       top_sample && sample_kth < k ? (const double*)th0 : (const double*)nullptr, b.thr0,
                       qc ? &qc[0].flag : (const float*)nullptr, (int)(sizeof(QConst) / 4), b,
                       queue_scan ? (const int*)flag_list : (const int*)nullptr,
                       queue_scan ? (const int*)flag_n : (const int*)nullptr);
    HQ_CHECK_LAUNCH();
  }
#ifdef HQ_DIAG
  if (b.expt == 3) {
    unsigned long long h[7];
    HQ_CHECK_HIP(hipMemcpyAsync(h, dbg, sizeof(h), hipMemcpyDeviceToHost, s));
    HQ_CHECK_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "k_scan0f: waves %d, insert entries %llu, passing pairs %llu, list inserts %llu, filter passes "
            "%llu in %llu (u, r) iterations, pre-filter fired in %llu of %llu half-steps\n", b.nqb * b.nchunks, h[0],
            h[1], h[2], h[3], h[4], h[5], h[6]);
  }
  if (!f32) {
    int mg = Q < 4096 ? Q : 4096;
    hipLaunchKernelGGL(k_merge, dim3(mg), dim3(64), 0, s, b.ws_score, b.ws_id, (const double*)nullptr,
                       (const int64_t*)nullptr, b.nchunks, Q, k, out_score, out_id, (double*)nullptr,
                       (int64_t*)nullptr);
    HQ_CHECK_LAUNCH();
  }
#endif
  return HQ_OK;
}

// Split-f16 level-0 copies for the default scan: Z16 = (hi[32], lo[32]) of the level-0 segment
// zero-padded to 32 for the rows [0, round_up(N, 16) + kPad0), in the tiled fragment layout (z16_frag),
// and S32 = per-row (std, mean, msq, flag bits: 1 zero variance,
// 2 msq outside [2^-60, 2^60], 4 pad row) in SoA groups of 4 rows: group G = rows 4G .. 4G + 3 holds
// std[4], mean[4], msq[4], flags[4] (16 floats), for the rows [0, round_up(N, 4) + kPad0).  k_scan0f
// reads up to 31 rows past a step start.

// one (row, value) of the split level-0 copies (row r < z16_rows(N), value c < 32)
__device__ __forceinline__ void pack0_elem(const double* __restrict__ Z, const double* __restrict__ S, int64_t N,
                                           int Lp, int P0, int nseg, _Float16* __restrict__ Z16,
                                           float* __restrict__ S32, int64_t r, int c) {
    {
      const double z = (r < N && c < P0) ? Z[r * Lp + c] : 0.0;
      const _Float16 hi = (_Float16)z;
      const _Float16 lo = (_Float16)(z - (double)hi);
      const int64_t e = z16_elem(r, c);
      Z16[e] = hi;
      Z16[e + kZ16Lo] = lo;
    }
    if (c == 0 && r < pack0_rows(N)) {
      float* o = S32 + (r >> 2) * 16 + (r & 3);
      if (r < N) {
        const double* st = S + r * nseg * 4;
        const double sd = st[1], mean = st[0], msq = st[2];
        int flag = sd == 0.0 ? 1 : 0;
        if (!(msq >= 0x1p-60 && msq <= 0x1p60)) flag |= 2;
        o[0] = (float)sd; o[4] = (float)mean; o[8] = (float)msq; o[12] = __int_as_float(flag);
      } else {
        o[0] = 0.0f; o[4] = 0.0f; o[8] = 1.0f; o[12] = __int_as_float(4);
      }
    }
}

__global__ void k_pack0(const double* __restrict__ Z, const double* __restrict__ S, int64_t N, int Lp, int P0,
                        int nseg, _Float16* __restrict__ Z16, float* __restrict__ S32) {
  const int64_t rows = z16_rows(N);  // >= pack0_rows(N)
  const int64_t total = rows * 32;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x)
    pack0_elem(Z, S, N, Lp, P0, nseg, Z16, S32, t / 32, (int)(t % 32));
}

// Query batches: k_seg_prepare_lds and k_pack0 in one launch (one wave per row: the row's segments, then
// its split level-0 copy from the Z / S the wave just wrote; blocks past N write the pad rows), the same
// arithmetic as the two kernels
__global__ __launch_bounds__(64) void k_seg_prepare_pack0(const double* __restrict__ idx, int64_t N, SegInfo si,
                                                          int all_f32, const uint8_t* __restrict__ row_f32,
                                                          double* __restrict__ Z, double* __restrict__ stats,
                                                          _Float16* __restrict__ Z16, float* __restrict__ S32) {
  extern __shared__ double xs[];  // L values
  const int lane = threadIdx.x;
  const int64_t rows = z16_rows(N);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    if (row < N) {
      for (int i = lane; i < si.L; i += 64) xs[i] = idx[row * si.L + i];
      __syncthreads();
      for (int sg = lane; sg < si.nseg; sg += 64) seg_prepare_one(xs, row, sg, si, all_f32, row_f32, Z, stats);
      __threadfence_block();
      __syncthreads();
    }
    if (lane < 32) pack0_elem(Z, stats, N, si.Lp, si.plen[0], si.nseg, Z16, S32, row, lane);
    __syncthreads();
  }
}

// Query batches, lane-cooperative (every level segment <= 128 values, at most 8 segments): one wave per row,
// each level segment's NumPy statistics summed by an 8-lane group (coop_sum: lane j owns the pairwise
// accumulator r_j) and its normalised values written by the group's lanes (m / 8 divisions each), then the
// split level-0 copy as k_seg_prepare_pack0.  The serial form has one lane walk each segment three times and
// divide every value.  Same operations as seg_prepare_one, so bit-identical.
__device__ __forceinline__ void seg_prepare_coop(const double* xrow, int64_t row, int s, const SegInfo& si,
                                                 int all_f32, const uint8_t* __restrict__ row_f32,
                                                 double* __restrict__ Z, double* __restrict__ stats, int j) {
  const double* x = xrow + si.src[s];
  const int m = si.len[s], plen = si.plen[s];
  const double mean = coop_sum<double>([=](int k) -> double { return x[k]; }, m, j) / (double)m;            // np.mean
  const double sd = sqrt(coop_sum<double>([=](int k) -> double { const double d = x[k] - mean; return d * d; }, m, j) /
                         (double)m);                                                                        // np.std
  const double msq = coop_sum<double>([=](int k) -> double { return x[k] * x[k]; }, m, j) / (double)m;      // mean(q**2)
  double* z = Z + row * si.Lp + si.poff[s];
  double* st = stats + (row * si.nseg + s) * 4;
  if (row_f32 ? row_f32[row] != 0 : all_f32 != 0) {
    const float mean32 = coop_sum<float>([=](int k) -> float { return (float)x[k]; }, m, j) / (float)m;
    const float sd32 = sqrtf(coop_sum<float>([=](int k) -> float { const float d = (float)x[k] - mean32; return d * d; },
                                             m, j) / (float)m);
    int aux = kAuxF32;
    if (!(msq >= 0x1p-100 && msq <= 0x1p100)) aux |= kAuxUnsafe;
    for (int i = j; i < plen; i += 8) z[i] = (sd32 == 0.0f || i >= m) ? 0.0 : (double)(((float)x[i] - mean32) / sd32);
    if (j == 0) {
      st[0] = sd32 == 0.0f ? (double)mean32 : mean;
      st[1] = (double)sd32;
      st[2] = msq;
      st[3] = (double)aux;
    }
    return;
  }
  for (int i = j; i < plen; i += 8) z[i] = (sd == 0.0 || i >= m) ? 0.0 : (x[i] - mean) / sd;
  if (j == 0) {
    st[0] = mean;
    st[1] = sd;
    st[2] = msq;
    st[3] = 0.0;
  }
}

__global__ __launch_bounds__(64) void k_seg_prepare_pack0_coop(const double* __restrict__ idx, int64_t N, SegInfo si,
                                                               int all_f32, const uint8_t* __restrict__ row_f32,
                                                               double* __restrict__ Z, double* __restrict__ stats,
                                                               _Float16* __restrict__ Z16, float* __restrict__ S32) {
  extern __shared__ double xs[];  // L values
  const int lane = threadIdx.x, gi = lane >> 3, j = lane & 7;
  const int64_t rows = z16_rows(N);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    if (row < N) {
      for (int i = lane; i < si.L; i += 64) xs[i] = idx[row * si.L + i];
      __syncthreads();
      for (int sg = gi; sg < si.nseg; sg += 8) seg_prepare_coop(xs, row, sg, si, all_f32, row_f32, Z, stats, j);
      __threadfence_block();
      __syncthreads();
    }
    if (lane < 32) pack0_elem(Z, stats, N, si.Lp, si.plen[0], si.nseg, Z16, S32, row, lane);
    __syncthreads();
  }
}

template <int KSMAX, bool OVERALL>
static int launch_scan(const ScanArgs& a, hipStream_t s) {
  const size_t lds = scan_lds_bytes(a.rs, a.nseg_used, a.K);
  HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_scan<KSMAX, OVERALL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
  const int grid = a.nqb * a.nchunks;
  hipLaunchKernelGGL((k_scan<KSMAX, OVERALL>), dim3(grid), dim3(256), lds, s, a);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

// exact re-rank launcher: the LDS-staged kernel when the staged rows fit (<= 96 KiB), else k_refine
// (which has no re-score output: odet then takes hq_rescore's kernel afterwards)
static int refine_launch(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                         const double* Zc, const double* Sc, int64_t N, int L, int mode, const double* cand_score,
                         const int64_t* cand_id, int kp, int k, double threshold, int thr_mode, double eps,
                         int64_t id_base, double* out_score, int64_t* out_id, int* out_count, int* out_resolved,
                         int count_empty, int* out_redo, double* out_det, hq_stream_t stream,
                         int* next_redo = nullptr, void* workspace = nullptr, size_t workspace_bytes = 0,
                         const FinalOut* fin = nullptr) {
  SegInfo si;
  seg_info(L, si);
  const hipStream_t s = (hipStream_t)stream;
  const int grid = Q < 8192 ? Q : 8192;
  // next_redo (hq_refine_rescore_topk_pp): out_redo arrives zeroed (cleared by the previous batch's kernel),
  // the kernel clears next_redo for the next batch; otherwise one 4-byte memset here
  if (out_redo && !next_redo) HQ_CHECK_HIP(hipMemsetAsync(out_redo, 0, sizeof(int), s));
  const bool sm = seg_small(si);
  auto rank_args = [&]() {
    RankArgs ra;
    ra.Rq = Rq; ra.Zq = Zq; ra.Sq = Sq; ra.Q = Q; ra.Rc = Rc; ra.Sc = Sc; ra.N = N;
    ra.cs.nseg = si.nseg; ra.cs.L = si.L; ra.cs.Lp = si.Lp;
    for (int i = 0; i < kCoopMaxW - 1; ++i) {
      ra.cs.src[i] = i < si.nseg ? si.src[i] : 0;
      ra.cs.len[i] = i < si.nseg ? si.len[i] : 0;
      ra.cs.poff[i] = i < si.nseg ? si.poff[i] : 0;
    }
    ra.mode = mode; ra.kp = kp; ra.k = k; ra.thr_mode = thr_mode; ra.det = out_det ? 1 : 0; ra.thr = threshold;
    ra.id_base = id_base; ra.cid = cand_id;
    ra.ws_sc = nullptr; ra.ws_id = nullptr; ra.ws_rec = nullptr;
    ra.win = (int)opt(OPT_RANK_WIN, 1);
    return ra;
  };
  // short lists: the fused lane-cooperative re-rank (k_rank_small) where its shapes hold; option
  // refine_small = 0 keeps k_refine_lds below (A/B, parity)
  if (kp <= kMaxTopK && coop_ppl(si) && opt(OPT_REFINE_SMALL, 1) != 0) {
    const RankArgs ra = rank_args();
    const int ng = kp <= 32 ? 32 : 64, W = 1 + si.nseg;
    const size_t lds = 8 * ((size_t)coop_qw(ra.cs) + (size_t)ng * coop_rw(ra.cs) + (size_t)ng * (2 + W)) + 8 * (size_t)ng;
    const FinalOut fo = fin ? *fin : FinalOut{0, nullptr, nullptr, nullptr, 0};
    double* odet_s = fin ? nullptr : out_det;
    const int ppl = coop_ppl(si);
    const void* fn = ng == 32 ? (ppl == 6 ? (const void*)k_rank_small<6, 32> : (const void*)k_rank_small<10, 32>)
                              : (ppl == 6 ? (const void*)k_rank_small<6, 64> : (const void*)k_rank_small<10, 64>);
    if (lds > 65536) HQ_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int c = count_empty ? 1 : 0;
    // compile-time level structures (L = 64, 32) here only with option rank_ct 2: at the 128-VGPR cap of this
    // kernel the unrolled scorer spills (28 VGPRs for L = 64)
    const int lid = ppl == 6 && opt(OPT_RANK_CT, 1) == 2 ? coop_lid(ra.cs) : 0;
    if (lid == 1 && ng == 32)
      hipLaunchKernelGGL((k_rank_small<6, 32, 1>), dim3(grid), dim3(256), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (lid == 2 && ng == 32)
      hipLaunchKernelGGL((k_rank_small<6, 32, 2>), dim3(grid), dim3(256), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (lid == 1)
      hipLaunchKernelGGL((k_rank_small<6, 64, 1>), dim3(grid), dim3(512), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (lid == 2)
      hipLaunchKernelGGL((k_rank_small<6, 64, 2>), dim3(grid), dim3(512), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (ng == 32 && ppl == 6)
      hipLaunchKernelGGL((k_rank_small<6, 32>), dim3(grid), dim3(256), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (ng == 32)
      hipLaunchKernelGGL((k_rank_small<10, 32>), dim3(grid), dim3(256), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else if (ppl == 6)
      hipLaunchKernelGGL((k_rank_small<6, 64>), dim3(grid), dim3(512), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    else
      hipLaunchKernelGGL((k_rank_small<10, 64>), dim3(grid), dim3(512), lds, s, ra, cand_score, eps, out_score, out_id,
                         out_count, out_resolved, c, out_redo, odet_s, next_redo, fo);
    HQ_CHECK_LAUNCH();
    return HQ_OK;
  }
  if (kp > kMaxTopK) {  // long lists: rows read from global memory, one workgroup per query
    // with a workspace (hq_refine_topk_ws): the lane-cooperative pair scoring (k_rank_pairs: 8 lanes per
    // entry, rows staged per group, every level in one pass) + the per-query ranking (k_rank_sort) where
    // its shapes hold; option refine_coop = 0 keeps the one-thread-per-entry kernels below (A/B, parity)
    const int ppl = coop_ppl(si);
    if (workspace && ppl && opt(OPT_REFINE_COOP, 1) != 0 && Q <= 65535) {
      if (workspace_bytes < refine_ws_bytes(Q, kp, L)) return fail(HQ_E_INVALID, "workspace too small");
      RankArgs ra = rank_args();
      uint8_t* w = reinterpret_cast<uint8_t*>(workspace);
      ra.ws_sc = reinterpret_cast<double*>(w);
      ra.ws_id = reinterpret_cast<int64_t*>(w + (size_t)Q * kp * 8);
      ra.ws_rec = reinterpret_cast<double*>(w + (size_t)Q * kp * 16);
      const size_t lds = 8 * ((size_t)coop_qw(ra.cs) + (size_t)kCoopGroups * coop_rw(ra.cs));
      // (round 6: two or four entries per group with the next row in flight measured 5-10% slower at M = 100 /
      // 1000 — profiles/r06_ab_count_read.txt, rank_e rows — the kernel was dropped)
      {
        const dim3 g1((kp + kCoopGroups - 1) / kCoopGroups, Q);
        const int lid = ppl == 6 ? coop_lid(ra.cs) : 0;  // compile-time level structures (L = 64, 32)
        if (lid == 1) hipLaunchKernelGGL((k_rank_pairs<6, 1>), g1, dim3(256), lds, s, ra);
        else if (lid == 2) hipLaunchKernelGGL((k_rank_pairs<6, 2>), g1, dim3(256), lds, s, ra);
        else if (ppl == 6) hipLaunchKernelGGL(k_rank_pairs<6>, g1, dim3(256), lds, s, ra);
        else hipLaunchKernelGGL(k_rank_pairs<10>, g1, dim3(256), lds, s, ra);
      }
      HQ_CHECK_LAUNCH();
      const FinalOut fo = fin ? *fin : FinalOut{0, nullptr, nullptr, nullptr, 0};
      double* od = fin ? nullptr : out_det;
      const int ce = count_empty ? 1 : 0;
      // lists > 512: 256 threads, four entries each (4 queries per CU at 118 VGPRs: M = 1000 1.70 -> 1.76M QPS,
      // profiles/r06_ab_rank_win.txt); option rank_sort_nt 512: one compare-exchange per thread and stage
      if (pow2_at_least(kp) <= 128 && opt(OPT_RANK_SORT_SMALL, 1) != 0)
        hipLaunchKernelGGL((k_rank_sort<128, 128>), dim3(grid), dim3(128), 0, s, ra, cand_score, eps, out_score,
                           out_id, out_count, out_resolved, ce, out_redo, od, next_redo, fo);
      else if (kp > 512 && opt(OPT_RANK_SORT_NT, 256) == 512)
        hipLaunchKernelGGL(k_rank_sort<512>, dim3(grid), dim3(512), 0, s, ra, cand_score, eps, out_score, out_id,
                           out_count, out_resolved, ce, out_redo, od, next_redo, fo);
      else
        hipLaunchKernelGGL(k_rank_sort<256>, dim3(grid), dim3(256), 0, s, ra, cand_score, eps, out_score, out_id,
                           out_count, out_resolved, ce, out_redo, od, next_redo, fo);
      HQ_CHECK_LAUNCH();
      return HQ_OK;
    }
    // lists of >= 512: the candidates' raw rows only (refine_big_body's ZB)
    const bool raw = kp >= 512;
    auto kern = sm ? (raw ? k_refine_big_sm_raw : k_refine_big_sm) : (raw ? k_refine_big_raw : k_refine_big);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc}, N, si, mode,
                       cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, out_score, out_id, out_count,
                       out_resolved, count_empty ? 1 : 0, out_redo, out_det, 0, next_redo, 0);
    HQ_CHECK_LAUNCH();
    return HQ_OK;
  }
  const size_t lds = ((size_t)refine_qw(si) + (size_t)kp * refine_rw(si) + (size_t)kp * (1 + si.nseg)) * 8;
#ifdef HQ_DIAG
  const int expt = (int)opt(OPT_REFINE_EXPT, 0);  // diagnostics build only
#else
  const int expt = 0;
#endif
  if (lds <= 96 * 1024 && L % 2 == 0 && !opt_on(OPT_REFINE_GLOBAL)) {  // 16-B pieces: L even
    const void* fn = sm ? (const void*)k_refine_lds_sm : (const void*)k_refine_lds;
    HQ_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (sm)
      hipLaunchKernelGGL(k_refine_lds_sm, dim3(grid), dim3(256), lds, s, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc},
                         N, si, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, out_score, out_id,
                         out_count, out_resolved, count_empty ? 1 : 0, out_redo, out_det, expt, next_redo);
    else
      hipLaunchKernelGGL(k_refine_lds, dim3(grid), dim3(256), lds, s, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc},
                         N, si, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, out_score, out_id,
                         out_count, out_resolved, count_empty ? 1 : 0, out_redo, out_det, expt, next_redo);
    HQ_CHECK_LAUNCH();
    return HQ_OK;
  }
  if (sm)
    hipLaunchKernelGGL(k_refine<true>, dim3(grid), dim3(64), 0, s, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc}, N, si,
                       mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, out_score, out_id, out_count,
                       out_resolved, count_empty ? 1 : 0, out_redo, next_redo);
  else
    hipLaunchKernelGGL(k_refine<false>, dim3(grid), dim3(64), 0, s, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc}, N, si,
                       mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, out_score, out_id, out_count,
                       out_resolved, count_empty ? 1 : 0, out_redo, next_redo);
  HQ_CHECK_LAUNCH();
  if (out_det) return hq_rescore(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, out_id, k, id_base, out_det, stream);
  return HQ_OK;
}


// ================================================================================================
// Overall-mode scan (brute_force_search, search_engine.py:302-338, scoring every candidate with
// _calculate_overall_similarity :191-230): the approximate overall score of every (query, row) pair
// from split-f16 contractions of every level segment, per-query pools as in k_scan0g, and the exact
// re-rank (hq_refine_topk mode 1) on top.
//   Layout (hq_seg_packov_split): the segments of >= 2 values ("G segments": one contraction each)
//   are packed in order into K-blocks of 32 values without straddling a block (L = 64: [32 | 8, 3,
//   20]; L = 32: [16, 4, 11]); each block's normalised values are split hi / lo in the tiled
//   fragment layout of Z16 (a 16-row tile holds NKB x [hi 512 | lo 512] halves).  One-value segments
//   always take the reference's constant branch (np.std of one value is 0): they need their value
//   only.  Statistics Sov32 in groups of 4 rows: per one-value segment value[4] and row flags[4] (2: a
//   G segment's mean of squares outside [2^-60, 2^60], scored by k_scanov_flagged in f64; 4: pad row)
//   for the scan's per-step loads, then per row its record (std, mean, msq, zero-std flag) per G
//   segment for the drain (one 16-byte load per segment).
//   Query side: one masked copy of the block fragment per G segment (values outside the segment
//   zeroed), so each contraction D[row][query] is that segment's G alone.
//   Pre-filter per pair (an upper bound of the f32 model score): a G segment scores at most
//   be + max(G, 0) ia (k_scan0f's U(G) with sqrt(A^2 G^2 + B^2) <= A |G| + |B|: be = 0.35 + |B| /
//   (2 sqrt Q), ia = c1 + A / (2 sqrt Q); a zero-variance candidate scores 0.1 <= be; a zero-variance
//   query segment is bounded by be = 1, ia = 0), a one-value segment 1 when the two values are within
//   1e-6 plus f32 slack, else 0.  Pairs whose weighted bound reaches the query's threshold are queued
//   (per pair: the G of every segment) and drained 64 at a time: the f32 model score (k_scan0g's per
//   level; constant branches decided exactly from the f64 means) and the pool append.
// ================================================================================================
constexpr int kOvMaxG = 4, kOvMaxC = 2, kOvMaxKB = 2;
constexpr int kOvQW = 32;       // queries per wave of k_scanov (two 16-query blocks)
constexpr int kOvQCap = 64 + 64 * 4;  // LDS queue entries per wave (< 64 before a block adds <= 256)

struct OvLayout {
  int nseg, ng, nc, nkb, lid;
  int gseg[kOvMaxG], gkb[kOvMaxG], goff[kOvMaxG], gplen[kOvMaxG], gpoff[kOvMaxG];
  int cseg[kOvMaxC];
  float gw[kOvMaxG], gc1[kOvMaxG], gqa[kOvMaxG], cw[kOvMaxC];  // weight 1/(l+1), 0.35/m, 0.6/m
  float inv_w;  // 1 / sum of weights (f32 model)
};

// compile-time K-block of each G segment, per supported layout id
template <int LID> struct OvT;
// seg(kb, k): the G segment holding value k of K-block kb (segments start at multiples of 4, so a dot2 pair
// never straddles two; padding values are zero in both copies and may be attributed to either side)
template <> struct OvT<0> {  // L = 64: [32 | 8, 3, 20], one one-value segment
  static constexpr int NKB = 2, NG = 4, NC = 1;
  // LIN form: the K-block contracted once with per-segment scaled query values (LKB), and whether
  // K-block 0 holds segment 0 alone (its scaled contraction then seeds the linear sum)
  static constexpr int LKB = 1;
  static constexpr bool LC0 = true;
  static constexpr int kb(int i) { return i == 0 ? 0 : 1; }
  static constexpr int seg(int b, int k) { return b == 0 ? 0 : (k < 8 ? 1 : (k < 12 ? 2 : 3)); }
};
template <> struct OvT<1> {  // L = 32: [16, 4, 11], one one-value segment
  static constexpr int NKB = 1, NG = 3, NC = 1;
  static constexpr int LKB = 0;
  static constexpr bool LC0 = false;
  static constexpr int kb(int) { return 0; }
  static constexpr int seg(int, int k) { return k < 16 ? 0 : (k < 20 ? 1 : 2); }
};

static bool ov_layout(int L, OvLayout& o) {
  SegInfo si;
  seg_info(L, si);
  o.nseg = si.nseg;
  o.ng = o.nc = o.nkb = 0;
  o.lid = -1;
  if (si.nseg == 0) return false;
  int kb = 0, off = 0;
  for (int s = 0; s < si.nseg; ++s) {
    if (si.len[s] == 1) {
      if (o.nc == kOvMaxC) return false;
      o.cseg[o.nc] = s;
      o.cw[o.nc] = (float)si.w[s];
      ++o.nc;
      continue;
    }
    if (si.plen[s] > 32 || o.ng == kOvMaxG) return false;
    if (o.ng > 0 && off + si.plen[s] > 32) { ++kb; off = 0; }
    if (kb >= kOvMaxKB) return false;
    o.gseg[o.ng] = s; o.gkb[o.ng] = kb; o.goff[o.ng] = off; o.gplen[o.ng] = si.plen[s]; o.gpoff[o.ng] = si.poff[s];
    o.gw[o.ng] = (float)si.w[s];
    o.gc1[o.ng] = (float)(0.35 * si.inv_m[s]);
    o.gqa[o.ng] = (float)(0.6 * si.inv_m[s]);
    ++o.ng;
    off += si.plen[s];
  }
  if (o.ng == 0) return false;
  o.nkb = kb + 1;
  o.inv_w = (float)(1.0 / si.wsum);
  auto match = [&](int nkb, int ng, int nc, auto kbf) {
    if (o.nkb != nkb || o.ng != ng || o.nc != nc) return false;
    for (int i = 0; i < ng; ++i)
      if (o.gkb[i] != kbf(i)) return false;
    return true;
  };
  if (match(OvT<0>::NKB, OvT<0>::NG, OvT<0>::NC, [](int i) { return OvT<0>::kb(i); })) o.lid = 0;
  else if (match(OvT<1>::NKB, OvT<1>::NG, OvT<1>::NC, [](int i) { return OvT<1>::kb(i); })) o.lid = 1;
  return o.lid >= 0;
}

__host__ __device__ __forceinline__ int ov_gsize(int ng, int nc) { return 16 * ng + 4 * nc + 8; }
// in a statistics group: one-value segment ci at 4 ci, the row flags at 4 nc, the rows' bound offsets at
// 4 nc + 4, row r's record of G segment i at 4 nc + 8 + 4 (r ng + i)
__host__ __device__ __forceinline__ int ov_rec(int ng, int nc, int r, int i) { return 4 * nc + 8 + 4 * (r * ng + i); }
// hi fragment (8 halves, k = 8 g .. 8 g + 7) of K-block kb of a row; lo at + kZ16Lo
__host__ __device__ __forceinline__ int64_t ov_frag(int64_t row, int kb, int nkb, int g) {
  return ((row >> 4) * nkb + kb) * kZ16Tile + ((g << 4) + (row & 15)) * 8;
}

__global__ void k_packov(const double* __restrict__ Z, const double* __restrict__ S, int64_t N, int Lp, OvLayout o,
                         _Float16* __restrict__ Zo, float* __restrict__ So) {
  const int64_t rows = z16_rows(N);
  const int per = o.nkb * 32;
  const int GS = ov_gsize(o.ng, o.nc);
  const int64_t total = rows * per;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / per;
    const int c = (int)(t % per), kb = c >> 5, k = c & 31;
    double z = 0.0;
    if (r < N)
      for (int i = 0; i < o.ng; ++i)
        if (o.gkb[i] == kb && k >= o.goff[i] && k < o.goff[i] + o.gplen[i]) z = Z[r * Lp + o.gpoff[i] + (k - o.goff[i])];
    const _Float16 hi = (_Float16)z;
    const _Float16 lo = (_Float16)(z - (double)hi);
    const int64_t e = ov_frag(r, kb, o.nkb, k >> 3) + (k & 7);
    Zo[e] = hi;
    Zo[e + kZ16Lo] = lo;
    if (c == 0 && r < pack0_rows(N)) {
      float* gp = So + (r >> 2) * GS;
      const int rr = (int)(r & 3);
      int flag = 4;
      float roff = 0.0f;
      if (r < N) {
        flag = 0;
        for (int i = 0; i < o.ng; ++i) {
          const double* st = S + (r * o.nseg + o.gseg[i]) * 4;
          const double mean = st[0], sd = st[1], msq = st[2];
          // a zero-variance segment scores 0.1 (or the query's constant branch), <= be - 0.25 (be >= 0.35)
          if (sd == 0.0) roff -= 0.25f * o.gw[i];
          float* rec = gp + ov_rec(o.ng, o.nc, rr, i);
          rec[0] = (float)sd;
          rec[1] = (float)mean;
          rec[2] = (float)msq;
          rec[3] = __int_as_float(sd == 0.0 ? 1 : 0);
          if (sd != 0.0 && !(msq >= 0x1p-60 && msq <= 0x1p60)) flag |= 2;
        }
        for (int ci = 0; ci < o.nc; ++ci) gp[4 * ci + rr] = (float)S[(r * o.nseg + o.cseg[ci]) * 4];
      } else {
        for (int i = 0; i < o.ng; ++i) {
          float* rec = gp + ov_rec(o.ng, o.nc, rr, i);
          rec[0] = 0.0f; rec[1] = 0.0f; rec[2] = 1.0f; rec[3] = __int_as_float(1);
        }
        for (int ci = 0; ci < o.nc; ++ci) gp[4 * ci + rr] = 0.0f;
      }
      gp[4 * o.nc + rr] = __int_as_float(flag);
      gp[4 * o.nc + 4 + rr] = roff;
    }
  }
}

// per-query constants of the overall scan (k_ov_qconst, from the query's Sov32 statistics and its
// starting threshold); QOvD: the model's part, cached in LDS by k_scanov
struct QOv {
  float thl, flag, wthr, bsum;         // pool threshold (f32 lower bound), flags, pre-filter bound, sum w be
  float wia[kOvMaxG], tolq[kOvMaxC], pad[2];  // pre-filter: w level <= w be + max(G, 0) w ia; one-value tolerance
  float qA[kOvMaxG], qB[kOvMaxG], qQ[kOvMaxG], qz[kOvMaxG];  // model constants; qz != 0: zero variance
  float cv[kOvMaxC], pad2[2];          // one-value segments: the query's value
};

struct QOvD {
  float qA[kOvMaxG], qB[kOvMaxG], qQ[kOvMaxG], qz[kOvMaxG];
  float cv[kOvMaxC], thl, pad;
};

__global__ void k_ov_qconst(const float* __restrict__ Sq, int Q, OvLayout o, const double* __restrict__ th0,
                            double thr0, QOv* __restrict__ qc) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  const int GS = ov_gsize(o.ng, o.nc);
  const float* gp = Sq + (int64_t)(q >> 2) * GS;
  const int rr = q & 3;
  QOv c;
  double t0 = thr0;
  if (th0 && th0[q] > t0) t0 = th0[q];
  c.thl = lower_f32(t0);
  c.flag = gp[4 * o.nc + rr];
  // pre-filter bound on the weighted sum, with slack for the f32 evaluation of bound and model
  c.wthr = t0 > -__builtin_huge_val() ? (c.thl - 1e-4f) / o.inv_w - 1e-4f : -__builtin_huge_valf();
  for (int i = 0; i < kOvMaxG; ++i) {
    c.wia[i] = 0.0f; c.qA[i] = 0.0f; c.qB[i] = 0.0f; c.qQ[i] = 1.0f; c.qz[i] = 1.0f;
  }
  c.bsum = 0.0f;
  c.pad[0] = c.pad[1] = 0.0f;
  for (int i = 0; i < o.ng; ++i) {
    const float* rec = gp + ov_rec(o.ng, o.nc, rr, i);
    const float sd = rec[0], mn = rec[1], ms = rec[2];
    const bool z = __float_as_int(rec[3]) != 0;
    c.qA[i] = o.gqa[i] * sd;
    c.qB[i] = 0.6f * mn;
    c.qQ[i] = ms;
    c.qz[i] = z ? 1.0f : 0.0f;
    float ia = 0.0f, be = 1.0f;
    if (!z) {
      const float h = 0.5f / sqrtf(ms);
      ia = (o.gc1[i] + c.qA[i] * h) * (1.0f + 1e-5f);
      be = (0.35f + fabsf(c.qB[i]) * h) * (1.0f + 1e-5f) + 1e-6f;
    }
    c.wia[i] = o.gw[i] * ia * (1.0f + 1e-6f);
    c.bsum += o.gw[i] * be * (1.0f + 1e-6f);
  }
  for (int ci = 0; ci < kOvMaxC; ++ci) {
    c.cv[ci] = ci < o.nc ? gp[4 * ci + rr] : 0.0f;
    c.tolq[ci] = 1e-6f + 2.5e-7f * fabsf(c.cv[ci]);
  }
  c.pad2[0] = c.pad2[1] = 0.0f;
  qc[q] = c;
}

// the f32 model overall score of one pair (G of each G segment given), or -1 when the row is not scored
// here (flagged: k_scanov_flagged; pad).  Constant branches are decided from the f64 means exactly as
// const0; the one-value segments compare the f32 values first and fall back to f64 near the edge.
// the reference's both-constant branch from the f64 means (out of line: rare)
__device__ __noinline__ float ov_const0(const double* __restrict__ sq, const double* __restrict__ sc) {
  return (float)const0(true, true, sq[0], sc[0], (aux_bits(sq) & aux_bits(sc) & kAuxF32) != 0);
}

template <int NG, int NC, class QC>
__device__ __forceinline__ float ov_model(const OvLayout& o, const QC& c, const float* __restrict__ Sc32, int64_t row,
                                          const float* G, const double* __restrict__ Sq, const double* __restrict__ Sc,
                                          int q) {
  constexpr int GS = 16 * NG + 4 * NC + 8;
  const float* gp = Sc32 + (row >> 2) * GS;
  const int rr = (int)(row & 3);
  if (__float_as_int(gp[4 * NC + rr]) != 0) return -1.0f;
  const double* sq = Sq + (int64_t)q * o.nseg * 4;
  const double* sc = Sc + row * o.nseg * 4;
  float tw = 0.0f;
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    float lvl;
    const flt4 rec = *reinterpret_cast<const flt4*>(gp + ov_rec(NG, NC, rr, i));  // std, mean, msq, zero-std
    const bool cz = __float_as_int(rec[3]) != 0, qz = c.qz[i] != 0.0f;
    if (qz || cz) {
      lvl = 0.1f;  // one side constant (search_engine.py:147-148)
      if (qz && cz) lvl = ov_const0(sq + 4 * o.gseg[i], sc + 4 * o.gseg[i]);
    } else {
      const float num = fmaf(G[i], c.qA[i] * rec[0], c.qB[i] * rec[1]);
      float t = num * __builtin_amdgcn_rcpf(c.qQ[i] + rec[2]);
      t = t > 0.0f ? t : 0.0f;
      lvl = fmaf(G[i], o.gc1[i], 0.35f) + t;
      lvl = lvl < 1.0f ? lvl : 1.0f;
      lvl = lvl > 0.0f ? lvl : 0.0f;
    }
    tw = fmaf(o.gw[i], lvl, tw);
  }
#pragma unroll
  for (int ci = 0; ci < NC; ++ci) {
    const float cv = gp[4 * ci + rr];
    const float d = fabsf(c.cv[ci] - cv), sl = 2.5e-7f * (fabsf(c.cv[ci]) + fabsf(cv)) + 1e-12f;
    float lvl;
    if (d > 1e-6f + sl) lvl = 0.0f;
    else if (d < 1e-6f - sl) lvl = 1.0f;
    else lvl = ov_const0(sq + 4 * o.cseg[ci], sc + 4 * o.cseg[ci]);
    tw = fmaf(o.cw[ci], lvl, tw);
  }
  float s = tw * o.inv_w;
  s = s < 1.0f ? s : 1.0f;
  return s > 0.0f ? s : 0.0f;
}

struct OvArgs {
  const _Float16* Zq; const float* Sq32; const double* Sq; int Q;
  const _Float16* Zc; const float* Sc32; const double* Sc; int64_t N;
  OvLayout o;
  const QOv* qc;
  int64_t chunk_len; int nchunks; int nqb;
  float* pool_s; int* pool_i; int* pool_n; int pool_cap;
  int64_t stride, S; float* top;  // sample pass
  const double* Zq64; const double* Zc64; int Lp;  // k_scanov_flagged: the f64 normalised vectors
};


// masked query fragments of one 16-query block: hi / lo of G segment i, values outside it zeroed
template <class T>
__device__ __forceinline__ void ov_query_frags(const OvArgs& a, int q, int g, half8* qh, half8* ql) {
#pragma unroll
  for (int i = 0; i < T::NG; ++i) {
    const _Float16* zr = a.Zq + ov_frag(q, T::kb(i), T::NKB, g);
    half8 h = *reinterpret_cast<const half8*>(zr);
    half8 l = *reinterpret_cast<const half8*>(zr + kZ16Lo);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * g + e;
      if (k < a.o.goff[i] || k >= a.o.goff[i] + a.o.gplen[i]) {
        h[e] = (_Float16)0.0f;
        l[e] = (_Float16)0.0f;
      }
    }
    qh[i] = h;
    ql[i] = l;
  }
}

// the split G (hi.hi + hi.lo + lo.hi, f32 accumulation by v_dot2_f32_f16) of every G segment of query q
// against one row of the overall layout: k_scanov's drain (its pre-filter contracted hi.hi only)
template <class T>
__device__ __forceinline__ void ov_split_g(const _Float16* __restrict__ Zq, const _Float16* __restrict__ Zc, int q,
                                           int64_t row, float* G) {
  float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f, g3 = 0.0f;
#pragma unroll 1
  for (int t = 0; t < 4 * T::NKB; ++t) {  // one k-group (8 values) at a time: few live VGPRs
    const int kb = t >> 2, gg = t & 3;
    const _Float16* pq = Zq + ov_frag(q, kb, T::NKB, gg);
    const _Float16* pc = Zc + ov_frag(row, kb, T::NKB, gg);
    const half8 qhv = *reinterpret_cast<const half8*>(pq), qlv = *reinterpret_cast<const half8*>(pq + kZ16Lo);
    const half8 chv = *reinterpret_cast<const half8*>(pc), clv = *reinterpret_cast<const half8*>(pc + kZ16Lo);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float d = __builtin_amdgcn_fdot2(h2(qhv, p), h2(chv, p), 0.0f, false);
      d = __builtin_amdgcn_fdot2(h2(qhv, p), h2(clv, p), d, false);
      d = __builtin_amdgcn_fdot2(h2(qlv, p), h2(chv, p), d, false);
      const int i = T::seg(kb, 8 * gg + 2 * p);  // partial sums of a pair's six products, then per segment
      g0 += i == 0 ? d : 0.0f;
      g1 += i == 1 ? d : 0.0f;
      g2 += i == 2 ? d : 0.0f;
      g3 += i == 3 ? d : 0.0f;
    }
  }
  G[0] = g0;
  if (T::NG > 1) G[1] = g1;
  if (T::NG > 2) G[2] = g2;
  if (T::NG > 3) G[3] = g3;
}

// max(x, 0) in one instruction (fmaxf adds a canonicalising v_max of x with itself).  A builtin, not
// inline asm: the hazard recognizer does not see an asm statement's reads, and a VALU read of an MFMA
// result needs wait states (an asm v_max right after the MFMA read the stale register).
__device__ __forceinline__ float relu_f32(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 3.0e38f); }

// weighted pre-filter bound of the lane's four rows (r) for one query block: two VALU per G segment
// (weights folded into wia / bsum per query), four per one-value segment
template <class T>
__device__ __forceinline__ void ov_bound(const flt4* acc, const float* wia, float bsum, const OvLayout& o,
                                         const float* qv, const float* tolq, const flt4* cvv, const flt4 ro, float* U) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float u = bsum + ro[r];  // rows with zero-variance G segments: their smaller bound
#pragma unroll
    for (int i = 0; i < T::NG; ++i) u = fmaf(relu_f32(acc[i][r]), wia[i], u);
#pragma unroll
    for (int ci = 0; ci < T::NC; ++ci) {
      const float d = fabsf(qv[ci] - cvv[ci][r]);
      const float uc = u + o.cw[ci];
      u = d <= fmaf(2.5e-7f, fabsf(cvv[ci][r]), tolq[ci]) ? uc : u;
    }
    U[r] = u;
  }
}

// One wave = 32 queries (two blocks b of 16; lane (g, j) owns queries 16b + j) x one chunk, 16 rows per
// step (lane group g owns rows 4g + r: the MFMA D layout), NG MFMAs (HI: hi.hi only) or NG x 3 (split) per
// block and step.  HI: the bound takes G_hihi, each segment's slack |G_split - G_hihi| < 1e-3 m + 1e-4 (as
// k_scan0g) folded into bsum (relu(G + d) <= relu(G) + d), and the drain recomputes the split G of every
// queued pair (ov_split_g) for the model score; the queue then holds the (row, query) key only.
//
// LIN (default with HI): the weighted relu sum in two parts, w relu(G) = s (G + |G|) with s = w ia / 2
// per segment and query.  The query's masked copies are pre-scaled by s in f16 (acc_i = s_i G_i), one
// more contraction of the shared K-block with per-segment scaled values (seeded with K-block 0's
// acc_0 when that block holds segment 0 alone) gives the linear part sum_i s_i G_i, and the bound is
// acc_lin + ro + sum_i |acc_i|: one VALU add (abs source modifier) per segment and pair instead of a
// med3 and an fma; the pair passes when it reaches the query's threshold less bsum and, per matching
// one-value segment, less its weight (A/B, cfg3 overall QPS: 0.88M vs 0.83M for the med3 + fma bound;
// a drain gate on the model at G_hihi + slack before the split measured slower, 0.69M, as did keeping
// G_hihi in the queue: the kernel is not bound by the drain's split recompute).  The f16 scaling errs by <= 2^-11 s_i sum|q c| <= 2^-11 s_i m_i
// in each part (Cauchy-Schwarz on unit-variance vectors), folded into bsum with the hi.hi slack.
template <int LID, int OCC, bool HI = true, bool LIN = HI, int PF = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OCC))) void k_scanov(OvArgs a) {
  using T = OvT<LID>;
  constexpr int NG = T::NG, NC = T::NC, NKB = T::NKB, NB = kOvQW / 16, GS = 16 * NG + 4 * NC + 8;
  __shared__ flt4 qg[HI ? 1 : kOvQCap];  // queue: G of each G segment (split form) ...
  __shared__ int qk[kOvQCap];   // ... and (row - c_begin) << 5 | query within the wave
  __shared__ QOvD qs[kOvQW];    // the wave's model constants (the drain reads them per entry)
  // LIN: pool appends collected in LDS and written after the scan loop, so the loop issues no global
  // store or atomic: on gfx9 the vector-memory counter is not ordered between loads and stores, and a
  // possibly pending store made every wait for the prefetched step a vmcnt(0) (the prefetch collapsed).
  // A wave whose buffer fills marks the queries it would drop as overflowing (dense path).
  constexpr int kAB = LIN ? 256 : 1;
  __shared__ float ab_s[kAB];
  __shared__ int ab_r[kAB];
  __shared__ unsigned int ab_over;
  int nab = 0;
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  if (lane == 0) ab_over = 0u;  // visible after the wave_lds_sync below
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  if (c_begin >= a.N) return;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.N) c_end = a.N;
  const int q0 = qb * kOvQW;
  const OvLayout& o = a.o;
  if (lane < kOvQW) {
    const QOv& c = a.qc[q0 + lane < a.Q ? q0 + lane : 0];
    QOvD d;
#pragma unroll
    for (int i = 0; i < kOvMaxG; ++i) { d.qA[i] = c.qA[i]; d.qB[i] = c.qB[i]; d.qQ[i] = c.qQ[i]; d.qz[i] = c.qz[i]; }
#pragma unroll
    for (int ci = 0; ci < kOvMaxC; ++ci) d.cv[ci] = c.cv[ci];
    d.thl = c.thl;
    d.pad = 0.0f;
    qs[lane] = d;
  }
  wave_lds_sync();

  static_assert(!LIN || HI, "the LIN bound is a hi.hi form");
  half8 qh[NB][NG], ql[HI ? 1 : NB][NG], qlin[LIN ? NB : 1];
  float wia[LIN ? 1 : NB][NG], bsum[NB], wt[NB], qv[NB][NC > 0 ? NC : 1], tolq[NB][NC > 0 ? NC : 1];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int q = q0 + 16 * b + j;
    const bool v = q < a.Q;
    const int qq = v ? q : 0;
    half8 lo_unused[NG];
    ov_query_frags<T>(a, qq, g, qh[b], HI ? lo_unused : ql[HI ? 0 : b]);
    const QOv& c = a.qc[qq];
    float wi[NG];
#pragma unroll
    for (int i = 0; i < NG; ++i) wi[i] = c.wia[i];
    if constexpr (!LIN) {
#pragma unroll
      for (int i = 0; i < NG; ++i) wia[b][i] = wi[i];
    }
    bsum[b] = c.bsum;
    if constexpr (HI) {
#pragma unroll
      for (int i = 0; i < NG; ++i) bsum[b] = fmaf(wi[i], 1e-3f * (float)o.gplen[i] + 1e-4f, bsum[b]);
    }
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) { qv[b][ci] = c.cv[ci]; tolq[b][ci] = c.tolq[ci]; }
    wt[b] = (v && __float_as_int(c.flag) == 0) ? c.wthr : __builtin_huge_valf();  // flagged query: dense path
    if constexpr (LIN) {
      // scaled copies: masked per segment (s_i q), and the shared K-block with each value scaled by its
      // segment's s; slack 2 x 2^-11 s_i m_i (both parts) + accumulation
      float sl = 0.0f;
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const float si = 0.5f * wi[i];
#pragma unroll
        for (int e = 0; e < 8; ++e) qh[b][i][e] = (_Float16)(si * (float)qh[b][i][e]);
        sl = fmaf(si, (float)o.gplen[i] * 1.0e-3f + 1e-5f, sl);
      }
      const _Float16* zr = a.Zq + ov_frag(qq, T::LKB, T::NKB, g);
      const half8 hv = *reinterpret_cast<const half8*>(zr);
      half8 lv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = T::seg(T::LKB, 8 * g + e);
        float si = 0.0f;
#pragma unroll
        for (int ii = 0; ii < NG; ++ii) si = ii == i ? 0.5f * wi[ii] : si;
        lv[e] = (_Float16)(si * (float)hv[e]);
      }
      qlin[b] = lv;
      bsum[b] += sl;
      wt[b] = wt[b] - bsum[b];  // the pair passes when acc_lin + sum |acc_i| (+ one-value terms) reach this
    }
  }

  const _Float16* zb = a.Zc + (c_begin >> 4) * NKB * kZ16Tile + lane * 8;
  const float* sb = a.Sc32 + (c_begin >> 2) * GS;  // one-value segment values of the step's first group
  struct CStep {
    half8 f[NKB][HI ? 1 : 2];
    flt4 cv[NC > 0 ? NC : 1];
    flt4 ro;
  };
  const int64_t nsteps = (c_end - c_begin + kCS - 1) / kCS;
  auto load_step = [&](CStep& c, int64_t s) {
    s = s < nsteps ? s : nsteps - 1;  // the prefetch stays inside the chunk
    const _Float16* p = zb + s * (NKB * kZ16Tile);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      c.f[kb][0] = *reinterpret_cast<const half8*>(p + kb * kZ16Tile);
      if constexpr (!HI) c.f[kb][HI ? 0 : 1] = *reinterpret_cast<const half8*>(p + kb * kZ16Tile + kZ16Lo);
    }
    const float* sp = sb + (s * 4 + g) * GS;
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) c.cv[ci] = *reinterpret_cast<const flt4*>(sp + 4 * ci);
    c.ro = *reinterpret_cast<const flt4*>(sp + 4 * NC + 4);
  };

  int qn = 0;
  // drain the first n <= 64 entries (one per lane): f32 model score, pool append; then shift the rest down
  auto drain = [&](const int n) {
    bool ok = false;
    float sv = 0.0f;
    int rk = 0;
    if (lane < n) {
      const int key = qk[lane], eqi = key & 31;
      const int64_t row = c_begin + (key >> 5);
      const int q = q0 + eqi;
      const QOvD& c = qs[eqi];
      if (row < c_end) {
        float G[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (HI) {
          ov_split_g<T>(a.Zq, a.Zc, q, row, G);
        } else {
          const flt4 eg = qg[lane];
#pragma unroll
          for (int i = 0; i < 4; ++i) G[i] = eg[i];
        }
        const float s = ov_model<NG, NC>(o, c, a.Sc32, row, G, a.Sq, a.Sc, q);
        if constexpr (LIN) {
          ok = s >= c.thl;
          sv = s;
          rk = (int)((row - c_begin) << 5) | eqi;
        } else if (s >= c.thl) {
          const int slot = atomicAdd(a.pool_n + q, 1);
          if (slot < a.pool_cap) {
            a.pool_s[(int64_t)q * a.pool_cap + slot] = s;
            a.pool_i[(int64_t)q * a.pool_cap + slot] = (int)row;
          }
        }
      }
    }
    if constexpr (LIN) {  // wave-uniform append position
      const unsigned long long m = __builtin_amdgcn_ballot_w64(ok);
      const int pos = nab + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (ok) {
        if (pos < kAB) {
          ab_s[pos] = sv;
          ab_r[pos] = rk;
        } else {
          atomicOr(&ab_over, 1u << (rk & 31));  // LDS atomic: no global memory traffic in the loop
        }
      }
      nab += __popcll(m);
      nab = nab < kAB ? nab : kAB;
    }
    wave_lds_sync();
    for (int b0 = n; b0 < qn; b0 += 64) {
      const bool mv = b0 + lane < qn;
      flt4 tg = {0.0f, 0.0f, 0.0f, 0.0f};
      int tk = 0;
      if (mv) {
        if constexpr (!HI) tg = qg[b0 + lane];
        tk = qk[b0 + lane];
      }
      wave_lds_sync();
      if (mv) {
        if constexpr (!HI) qg[b0 - n + lane] = tg;
        qk[b0 - n + lane] = tk;
      }
      wave_lds_sync();
    }
    qn -= n;
  };
  // one block of one step: contractions, bound, queue the passing pairs (drained once per step)
  auto block = [&](const int b, const CStep& cur, const int64_t cs) {
    flt4 acc[NG];
#pragma unroll
    for (int i = 0; i < NG; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cur.f[T::kb(i)][0], qh[b][i], flt4{0, 0, 0, 0}, 0, 0, 0);
    if constexpr (!HI) {
#pragma unroll
      for (int i = 0; i < NG; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cur.f[T::kb(i)][0], ql[HI ? 0 : b][i], acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NG; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cur.f[T::kb(i)][HI ? 0 : 1], qh[b][i], acc[i], 0, 0, 0);
    }
    float U[4], W[4];
    if constexpr (LIN) {
      const flt4 al = __builtin_amdgcn_mfma_f32_16x16x32_f16(cur.f[T::LKB][0], qlin[b], T::LC0 ? acc[0] : flt4{0, 0, 0, 0},
                                                              0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float u = al[r] + cur.ro[r];  // rows with zero-variance G segments: their smaller bound
#pragma unroll
        for (int i = 0; i < NG; ++i) u += fabsf(acc[i][r]);
        float t = wt[b];
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
          const float d = fabsf(qv[b][ci] - cur.cv[ci][r]);
          t = d <= fmaf(2.5e-7f, fabsf(cur.cv[ci][r]), tolq[b][ci]) ? t - o.cw[ci] : t;
        }
        U[r] = u;
        W[r] = t;
      }
    } else {
      ov_bound<T>(acc, wia[b], bsum[b], o, qv[b], tolq[b], cur.cv, cur.ro, U);
#pragma unroll
      for (int r = 0; r < 4; ++r) W[r] = wt[b];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned long long m = __builtin_amdgcn_ballot_w64(U[r] >= W[r]);
      if (m) {
        if ((m >> lane) & 1ull) {
          const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
          if constexpr (!HI) {
            flt4 gg = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int i = 0; i < NG; ++i) gg[i] = acc[i][r];
            qg[pos] = gg;
          }
          qk[pos] = (int)((cs - c_begin + 4 * g + r) << 5) | (16 * b + j);
        }
        qn += __popcll(m);
      }
    }
    if (qn >= 64) {  // keeps qn < 64 before each block: the queue never exceeds 63 + 4 x 64
      wave_lds_sync();
      while (qn >= 64) drain(64);
    }
  };
  auto step = [&](const CStep& cur, const int64_t s) {
#pragma unroll
    for (int b = 0; b < NB; ++b) block(b, cur, c_begin + s * kCS);
  };

  // LIN: the wave's pool appends, after its scan loop; queries whose appends did not fit the buffer get a
  // count past the pool capacity (k_pool_select then sends them to the dense exact path)
  auto flush = [&] {
    if constexpr (LIN) {
      wave_lds_sync();
      for (int e = lane; e < nab; e += 64) {
        const int rk2 = ab_r[e], eqi = rk2 & 31, q = q0 + eqi;
        const int slot = atomicAdd(a.pool_n + q, 1);
        if (slot < a.pool_cap) {
          a.pool_s[(int64_t)q * a.pool_cap + slot] = ab_s[e];
          a.pool_i[(int64_t)q * a.pool_cap + slot] = (int)(c_begin + (rk2 >> 5));
        }
      }
      const unsigned int over = ab_over;
      if (lane < 32 && ((over >> lane) & 1u) && q0 + lane < a.Q) atomicAdd(a.pool_n + q0 + lane, a.pool_cap + 1);
    }
  };
  if constexpr (PF == 1) {  // two buffers, ping-pong
    CStep cA, cB;
    load_step(cA, 0);
    int64_t s = 0;
    for (; s + 1 < nsteps; s += 2) {
      load_step(cB, s + 1);
      __builtin_amdgcn_sched_barrier(0);
      step(cA, s);
      load_step(cA, s + 2);
      __builtin_amdgcn_sched_barrier(0);
      step(cB, s + 1);
    }
    if (s < nsteps) step(cA, s);
    wave_lds_sync();
    while (qn > 0) drain(qn < 64 ? qn : 64);
    flush();
    return;
  }
  // PF + 1 step buffers in rotation: step s + PF is requested while step s is scored (load_step clamps
  // the index to the chunk's last step)
  CStep buf[PF + 1];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_step(buf[u], u);
  auto body = [&](const int64_t st, const CStep& cur, CStep& nn) {
    load_step(nn, st + PF);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch PF steps ahead
    step(cur, st);
  };
  int64_t s = 0;
  for (; s + PF < nsteps; s += PF + 1) {
#pragma unroll
    for (int u = 0; u <= PF; ++u) body(s + u, buf[u], buf[(u + PF) % (PF + 1)]);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (s + u < nsteps) step(buf[u], s + u);
  wave_lds_sync();
  while (qn > 0) drain(qn < 64 ? qn : 64);
  flush();
}

// Sample pass of the overall scan (as k_sample_topg): 16 queries per wave, whole sample tiles; per lane
// the step whose four rows hold the largest pre-filter bound is kept and its rows are scored with the
// model in the epilogue; the stream's kTopT best go to the pool for k_sample_kth.  HI (default): the step
// loop contracts hi.hi only (the kept step is a heuristic choice: any choice leaves the sample's scores real
// scores of distinct pairs) and the epilogue recomputes the kept rows' split G (ov_split_g) for the model.
template <int LID, bool HI = true>
__global__ __launch_bounds__(64) void k_sampleov(OvArgs a) {
  using T = OvT<LID>;
  constexpr int NG = T::NG, NC = T::NC, NKB = T::NKB, GS = 16 * NG + 4 * NC + 8;
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int blk = blockIdx.x, xcd = blk & 7, slot = blk >> 3;
  const int chunk = xcd + 8 * (slot / a.nqb);
  const int qb = slot % a.nqb;
  if (chunk >= a.nchunks) return;
  const int64_t c_begin = (int64_t)chunk * a.chunk_len;
  int64_t c_end = c_begin + a.chunk_len;
  if (c_end > a.S) c_end = a.S;
  const OvLayout& o = a.o;
  const int q = qb * 16 + j;
  const bool qv_ok = q < a.Q;
  const int qq = qv_ok ? q : 0;
  half8 qh[NG], ql[NG];
  ov_query_frags<T>(a, qq, g, qh, ql);
  const QOv c = a.qc[qq];
  auto row_of = [&](int64_t i) -> int64_t { return sample_row_tiled(i, a.S, a.stride); };
  auto load = [&](int64_t cs, half8 (*f)[2], flt4* cv, flt4& ro) {
    const int64_t row = row_of(cs + j);  // tile-aligned: the step is one corpus tile
    const _Float16* p = a.Zc + ov_frag(row, 0, NKB, g);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      f[kb][0] = *reinterpret_cast<const half8*>(p + kb * kZ16Tile);
      if constexpr (!HI) f[kb][1] = *reinterpret_cast<const half8*>(p + kb * kZ16Tile + kZ16Lo);
    }
    const int64_t r0 = row_of(cs + 4 * g);
    const float* sp = a.Sc32 + (r0 >> 2) * GS;
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) cv[ci] = *reinterpret_cast<const flt4*>(sp + 4 * ci);
    ro = *reinterpret_cast<const flt4*>(sp + 4 * NC + 4);
  };
  float bu = -__builtin_huge_valf();
  flt4 bg[NG];
  int bcs = -1;
#pragma unroll
  for (int i = 0; i < NG; ++i) bg[i] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
  half8 f0[NKB][2], f1[NKB][2];
  flt4 v0[NC > 0 ? NC : 1], v1[NC > 0 ? NC : 1], ro0, ro1;
  load(c_begin, f0, v0, ro0);
  for (int64_t cs = c_begin; cs < c_end; cs += kCS) {
    load(cs + kCS, f1, v1, ro1);
    flt4 acc[NG];
#pragma unroll
    for (int i = 0; i < NG; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f0[T::kb(i)][0], qh[i], flt4{0, 0, 0, 0}, 0, 0, 0);
    if constexpr (!HI) {
#pragma unroll
      for (int i = 0; i < NG; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f0[T::kb(i)][0], ql[i], acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NG; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f0[T::kb(i)][1], qh[i], acc[i], 0, 0, 0);
    }
    float U[4];
    ov_bound<T>(acc, c.wia, c.bsum, o, c.cv, c.tolq, v0, ro0, U);
    float m = -__builtin_huge_valf();
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (cs + 4 * g + r < c_end) m = fmaxf(m, U[r]);
    const bool up = m > bu;
    bu = up ? m : bu;
    bcs = up ? (int)cs : bcs;
#pragma unroll
    for (int i = 0; i < NG; ++i) bg[i] = up ? acc[i] : bg[i];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      f0[kb][0] = f1[kb][0];
      if constexpr (!HI) f0[kb][1] = f1[kb][1];
    }
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) v0[ci] = v1[ci];
    ro0 = ro1;
  }
  if (!qv_ok) return;
  float top[kTopT];
#pragma unroll
  for (int t = 0; t < kTopT; ++t) top[t] = -1.0f;
  if (__float_as_int(c.flag) == 0 && bcs >= 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t i = (int64_t)bcs + 4 * g + r;
      if (i >= c_end) continue;
      float G[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (HI) {
        ov_split_g<T>(a.Zq, a.Zc, q, row_of(i), G);
      } else {
#pragma unroll
        for (int s = 0; s < NG; ++s) G[s] = bg[s][r];
      }
      float sc = ov_model<NG, NC>(o, c, a.Sc32, row_of(i), G, a.Sq, a.Sc, q);
      if (sc < 0.0f) continue;
#pragma unroll
      for (int u = 0; u < kTopT; ++u) {
        const float hi = fmaxf(top[u], sc);
        sc = fminf(top[u], sc);
        top[u] = hi;
      }
    }
  }
  float* out = a.top + ((int64_t)q * 4 * a.nchunks + 4 * chunk + g) * kTopT;
#pragma unroll
  for (int t = 0; t < kTopT; ++t) out[t] = top[t];
}

// rows of the overall copies with the f32-unsafe flag (row flags bit 2), compacted into list[*count]
__global__ __launch_bounds__(256) void k_ov_flag_rows(const float* __restrict__ So, int64_t N, int GS, int foff,
                                                      int* __restrict__ list, int* __restrict__ count) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x)
    if (__float_as_int(So[(r >> 2) * GS + foff + (r & 3)]) & 2) list[atomicAdd(count, 1)] = (int)r;  // foff = 4 nc
}

// the flagged rows against every scanned query (lane = query): the overall score in f64 from the f64
// normalised vectors (level_sim per segment), appended to the pools when it reaches the threshold
__global__ __launch_bounds__(64) void k_scanov_flagged(OvArgs a, SegInfo si, const int* __restrict__ list,
                                                       const int* __restrict__ count) {
  const int n = *count;
  const int q = blockIdx.y * 64 + threadIdx.x;
  if (q >= a.Q || n == 0) return;
  const QOv c = a.qc[q];
  if (__float_as_int(c.flag) != 0) return;
  const double* sq = a.Sq + (int64_t)q * si.nseg * 4;
  const double* zq = a.Zq64 + (int64_t)q * a.Lp;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int row = list[i];
    const double* sc = a.Sc + (int64_t)row * si.nseg * 4;
    const double* zc = a.Zc64 + (int64_t)row * a.Lp;
    double tws = 0.0;
    for (int s = 0; s < si.nseg; ++s) {
      double G = 0.0;
      for (int k = si.poff[s]; k < si.poff[s] + si.plen[s]; ++k) G = fma(zq[k], zc[k], G);
      const double v = level_sim(G, sq[4 * s], sq[4 * s + 1], sq[4 * s + 2], sc[4 * s], sc[4 * s + 1], sc[4 * s + 2],
                                 (double)si.len[s], si.inv_m[s], (aux_bits(sq + 4 * s) & aux_bits(sc + 4 * s) & kAuxF32) != 0);
      tws = tws + v * si.w[s];
    }
    double ov = tws / si.wsum;
    ov = ov < 1.0 ? ov : 1.0;
    ov = ov > 0.0 ? ov : 0.0;
    const float sv = (float)ov;
    if (sv >= c.thl) {
      const int slot = atomicAdd(a.pool_n + q, 1);
      if (slot < a.pool_cap) {
        a.pool_s[(int64_t)q * a.pool_cap + slot] = sv;
        a.pool_i[(int64_t)q * a.pool_cap + slot] = row;
      }
    }
  }
}

// grid of k_scanov / k_sampleov: ~waves waves of qw queries, chunks a multiple of 8 (XCD map) and of 16 rows
static void ov_geometry(int Q, int64_t rows, int qw, int waves, int max_chunks, int& nqb, int& nchunks,
                        int64_t& chunk_len) {
  nqb = (Q + qw - 1) / qw;
  int64_t target = (waves + nqb - 1) / nqb;
  const int64_t steps = (rows + kCS - 1) / kCS;
  if (target > steps) target = steps;
  if (target > max_chunks) target = max_chunks;
  nchunks = (int)(((target + 7) / 8) * 8);
  if (nchunks < 8) nchunks = 8;
  chunk_len = (rows + nchunks - 1) / nchunks;
  chunk_len = ((chunk_len + kCS - 1) / kCS) * kCS;
  if (chunk_len < kCS) chunk_len = kCS;
}

struct OvPlan {
  int nqb, nchunks, s_nqb, s_nchunks;
  int64_t chunk_len, s_chunk_len, stride, S;
  int pool_cap;
  size_t off_pool_i, off_pool_n, off_th0, off_top, off_qc, off_flag, total;
};

static OvPlan ov_plan(int Q, int64_t N, int k) {
  OvPlan p;
  // one round of waves at the kernel's occupancy (the hi.hi form: 4 waves per SIMD, 128 VGPRs; option
  // ov_occ 2 / 3)
  const int occ = (int)opt(OPT_OV_OCC, 4) == 2 ? 2 : ((int)opt(OPT_OV_OCC, 4) == 3 ? 3 : 4);
  int w = opt(OPT_OV_WAVES, 0) > 0 ? (int)opt(OPT_OV_WAVES, 0) : 1024 * occ;
  ov_geometry(Q, N, kOvQW, w, 1 << 20, p.nqb, p.nchunks, p.chunk_len);
  while (p.chunk_len > (int64_t(1) << 26)) {  // queue keys hold (row - chunk start) << 5
    w *= 2;
    ov_geometry(Q, N, kOvQW, w, 1 << 20, p.nqb, p.nchunks, p.chunk_len);
  }
  const int64_t sd = opt(OPT_SAMPLE_STRIDE, 16) > 0 ? opt(OPT_SAMPLE_STRIDE, 16) : 16;
  p.stride = N >= sd * 4096 ? sd : (N / 4096 > 1 ? N / 4096 : 1);
  p.S = sample_rows_tiled(N, p.stride);
  ov_geometry(Q, p.S, 16, 4096, 64 * kKthReg / (4 * kTopT), p.s_nqb, p.s_nchunks, p.s_chunk_len);
  p.pool_cap = pool_cap_for(p.nchunks, k, N, p.stride, scan_kprime(k, p.stride));
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = al((size_t)Q * p.pool_cap * 4);
  p.off_pool_i = 0 + o;
  o = al(o + (size_t)Q * p.pool_cap * 4);
  p.off_pool_n = o;
  o = al(o + (size_t)Q * 4);
  p.off_th0 = o;
  o = al(o + (size_t)Q * 8);
  p.off_top = o;
  o = al(o + (size_t)Q * 4 * p.s_nchunks * kTopT * 4);
  p.off_qc = o;
  o = al(o + (size_t)Q * sizeof(QOv));
  p.off_flag = o;
  o = al(o + 256 + (size_t)N * 4);
  p.total = o;
  return p;
}

template <int LID>
static int ov_launch(const OvArgs& a0, const OvPlan& p, const SegInfo& si, int k, double thr0, int sample_kth,
                     int64_t id_base, uint8_t* ws, double* out_score, int64_t* out_id, hipStream_t s) {
  OvArgs a = a0;
  const int Q = a.Q;
  a.pool_cap = p.pool_cap;
  a.pool_s = reinterpret_cast<float*>(ws);
  a.pool_i = reinterpret_cast<int*>(ws + p.off_pool_i);
  a.pool_n = reinterpret_cast<int*>(ws + p.off_pool_n);
  double* th0 = reinterpret_cast<double*>(ws + p.off_th0);
  QOv* qc = reinterpret_cast<QOv*>(ws + p.off_qc);
  int* flag_n = reinterpret_cast<int*>(ws + p.off_flag);
  int* flag_list = flag_n + 64;
  a.qc = qc;
  // sample pass: per-query constants without a threshold, the G-selected sample, K'-th best
  hipLaunchKernelGGL(k_ov_qconst, dim3((Q + 255) / 256), dim3(256), 0, s, a.Sq32, Q, a.o, (const double*)nullptr,
                     -__builtin_huge_val(), qc);
  HQ_CHECK_LAUNCH();
  OvArgs sa = a;
  sa.stride = p.stride;
  sa.S = p.S;
  sa.nqb = p.s_nqb;
  sa.nchunks = p.s_nchunks;
  sa.chunk_len = p.s_chunk_len;
  sa.top = reinterpret_cast<float*>(ws + p.off_top);
  // the split sample by default: the hi.hi form's epilogue (split G of the kept rows) measured 139 vs 106 us
  if (opt(OPT_SAMPLE_HI, 0) == 1) hipLaunchKernelGGL((k_sampleov<LID, true>), dim3(sa.nqb * sa.nchunks), dim3(64), 0, s, sa);
  else hipLaunchKernelGGL((k_sampleov<LID, false>), dim3(sa.nqb * sa.nchunks), dim3(64), 0, s, sa);
  HQ_CHECK_LAUNCH();
  const int mg = Q < 8192 ? Q : 8192;
  launch_kth(mg, s, (const float*)sa.top, 4 * sa.nchunks, Q, sample_kth, (double)kMarginF, th0,
             (unsigned long long*)nullptr, a.pool_n, (const float*)nullptr, thr0, 0.0, (QConst*)nullptr);
  HQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ov_qconst, dim3((Q + 255) / 256), dim3(256), 0, s, a.Sq32, Q, a.o, (const double*)th0, thr0, qc);
  HQ_CHECK_LAUNCH();
  // flagged rows (normally none), the scan, the pools' exact top k
  HQ_CHECK_HIP(hipMemsetAsync(flag_n, 0, sizeof(int), s));
  const int64_t fb = (a.N + 255) / 256;
  const int GS = ov_gsize(a.o.ng, a.o.nc);
  hipLaunchKernelGGL(k_ov_flag_rows, dim3((unsigned)(fb < 4096 ? fb : 4096)), dim3(256), 0, s, a.Sc32, a.N, GS,
                     4 * a.o.nc, flag_list, flag_n);
  HQ_CHECK_LAUNCH();
  // default: the hi.hi form at 4 waves per SIMD (option ov_occ 2 / 3); option scanov_split3: the split form
  const int oocc = (int)opt(OPT_OV_OCC, 4);
  if (opt_on(OPT_SCANOV_SPLIT3)) {
    if (oocc == 3) hipLaunchKernelGGL((k_scanov<LID, 3, false>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((k_scanov<LID, 2, false>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else if (opt_on(OPT_SCANOV_V1) || k > kMaxTopK) {
    // the med3 + fma bound with pool appends straight to global memory: long lists (k > 64) pass more pairs
    // per wave than the LIN form's 256-entry LDS append buffer holds (its overflow sends queries to the
    // dense path)
    hipLaunchKernelGGL((k_scanov<LID, 4, true, false>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else if (opt(OPT_OV_PF, 1) == 2) {  // prefetch distance (steps)
    if (oocc == 3) hipLaunchKernelGGL((k_scanov<LID, 3, true, true, 2>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((k_scanov<LID, 4, true, true, 2>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else if (opt(OPT_OV_PF, 1) == 3) {
    if (oocc == 3) hipLaunchKernelGGL((k_scanov<LID, 3, true, true, 3>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((k_scanov<LID, 4, true, true, 3>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else if (oocc == 2) {
    hipLaunchKernelGGL((k_scanov<LID, 2>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else if (oocc == 3) {
    hipLaunchKernelGGL((k_scanov<LID, 3>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  } else {
    // (round 6: one ballot over a block's four rows before the per-row queueing — the rows' bound chains
    // independent — spilled at 4 waves per SIMD (873 -> 2420 us per 1000 x 1M scan) and measured 16% slower
    // at 3 (0.77 vs 0.91M QPS, no spill): profiles/r06_ab_rank_ct.txt, r06_ab_final_select.txt; not kept)
    hipLaunchKernelGGL((k_scanov<LID, 4>), dim3(a.nqb * a.nchunks), dim3(64), 0, s, a);
  }
  HQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_scanov_flagged, dim3(64, (Q + 63) / 64), dim3(64), 0, s, a, si, (const int*)flag_list,
                     (const int*)flag_n);
  HQ_CHECK_LAUNCH();
  launch_pool_select(k, s, Q, a.pool_s, a.pool_i, a.pool_n, a.pool_cap, id_base, out_score, out_id,
                     sample_kth < k ? (const double*)th0 : (const double*)nullptr, thr0, &qc[0].flag,
                     (int)(sizeof(QOv) / 4), Scan0Args{}, (const int*)nullptr, (const int*)nullptr);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_diag_violations(int64_t* count, int* first_line) {
  unsigned long long c = 0;
  int line = 0;
#ifdef HQ_DIAG
  HQ_CHECK_HIP(hipDeviceSynchronize());
  HQ_CHECK_HIP(hipMemcpyFromSymbol(&c, HIP_SYMBOL(g_diag_count), sizeof(c)));
  HQ_CHECK_HIP(hipMemcpyFromSymbol(&line, HIP_SYMBOL(g_diag_line), sizeof(line)));
#endif
  if (count) *count = (int64_t)c;
  if (first_line) *first_line = line;
  return HQ_OK;
}

int hq_scan0_geometry(int Q, int64_t N, int* nqb, int* nchunks, int64_t* chunk_len, int64_t* z_rows,
                      int64_t* s_rows) {
  if (Q <= 0 || N <= 0) return fail(HQ_E_INVALID, "bad shape Q=%d N=%lld", Q, (long long)N);
  int a = 0, b = 0;
  int64_t c = 0;
  scan0_geometry(Q, N, a, b, c, kQW, opt(OPT_SCAN_OCC, 3) == 3 ? 3 : 4);  // the default scan's geometry
  if (nqb) *nqb = a;
  if (nchunks) *nchunks = b;
  if (chunk_len) *chunk_len = c;
  if (z_rows) *z_rows = z16_rows(N);
  if (s_rows) *s_rows = pack0_rows(N);
  return HQ_OK;
}

int hq_seg_count(int L) {
  SegInfo si;
  seg_info(L, si);
  return si.nseg;
}

int hq_seg_padded_len(int L) {
  SegInfo si;
  seg_info(L, si);
  return si.Lp;
}

int hq_seg_prepare(const double* idx, int64_t N, int L, double* Z, double* stats, hq_stream_t stream) {
  return hq_seg_prepare_src(idx, N, L, 0, Z, stats, stream);
}

int hq_seg_prepare_src(const double* idx, int64_t N, int L, int src_f32, double* Z, double* stats,
                       hq_stream_t stream) {
  return hq_seg_prepare_rows(idx, N, L, src_f32, nullptr, Z, stats, stream);
}

int hq_seg_prepare_rows(const double* idx, int64_t N, int L, int src_f32, const uint8_t* row_f32, double* Z,
                        double* stats, hq_stream_t stream) {
  if (L <= 0 || N < 0) return fail(HQ_E_INVALID, "bad shape N=%lld L=%d", (long long)N, L);
  if (N == 0) return HQ_OK;
  if (!idx || !Z || !stats) return fail(HQ_E_INVALID, "null buffer");
  SegInfo si;
  seg_info(L, si);
  if (si.nseg == 0) return fail(HQ_E_INVALID, "no level structure for L=%d", L);
  const int64_t total = N * si.nseg;
  if (N <= 16384 && si.L <= 4096 && !opt_on(OPT_SEG_PREPARE_FLAT)) {  // A/B option: the flat kernel
    hipLaunchKernelGGL(k_seg_prepare_lds, dim3((unsigned)N), dim3(64), (size_t)8 * si.L, (hipStream_t)stream, idx, N,
                       si, src_f32 ? 1 : 0, row_f32, Z, stats);
  } else {
    int64_t blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_seg_prepare, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, idx, N, si,
                       src_f32 ? 1 : 0, row_f32, Z, stats);
  }
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_level_scores(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc, const double* Zc,
                    const double* Sc, int64_t N, int L, int level, double* scores, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || N == 0) return HQ_OK;
  if (!Rq || !Zq || !Sq || !Rc || !Zc || !Sc || !scores) return fail(HQ_E_INVALID, "null buffer");
  SegInfo si;
  seg_info(L, si);
  if (level >= 0 && level < si.nseg && si.len[level] <= 128 && !opt_on(OPT_LEVEL_SCORES_V1) &&
      (N + kLsTile - 1) / kLsTile < (int64_t(1) << 31) && (Q + kLsQ - 1) / kLsQ < 65536) {
    const size_t lds = (size_t)kLsTile * (si.len[level] | 1) * 8;
    // segments of 65..128 values stage up to 132 KB: above the 64 KB default, so opt in (one block per CU)
    if (lds > 65536)
      HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_level_scores_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
    hipLaunchKernelGGL(k_level_scores_lds, dim3((unsigned)((N + kLsTile - 1) / kLsTile), (Q + kLsQ - 1) / kLsQ),
                       dim3(kLsTile), lds, (hipStream_t)stream, VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc}, N, si, level,
                       scores);
    HQ_CHECK_LAUNCH();
    return HQ_OK;
  }
  const int64_t total = (int64_t)Q * N;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (seg_small(si))
    hipLaunchKernelGGL(k_level_scores<true>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, VecSet{Rq, Zq, Sq}, Q,
                     VecSet{Rc, Zc, Sc}, N, si, level, scores);
  else
    hipLaunchKernelGGL(k_level_scores<false>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, VecSet{Rq, Zq, Sq}, Q,
                     VecSet{Rc, Zc, Sc}, N, si, level, scores);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_refine_topk(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc, const double* Zc,
                   const double* Sc, int64_t N, int L, int mode, const double* cand_score, const int64_t* cand_id,
                   int kp, int k, double threshold, int thr_mode, double eps, int64_t id_base, double* out_score,
                   int64_t* out_id, int* out_count, int* out_resolved, int count_empty, int* out_redo,
                   hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || kp <= 0 || kp > kMaxTopKBig || k <= 0 || k > kp)
    return fail(HQ_E_INVALID, "bad sizes kp=%d k=%d", kp, k);
  if (Q == 0) return HQ_OK;
  if (!Rq || !Zq || !Sq || !cand_score || !cand_id || !out_score || !out_id || !out_count || !out_resolved ||
      (N > 0 && (!Rc || !Zc || !Sc)))
    return fail(HQ_E_INVALID, "null buffer");
  return refine_launch(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps,
                       id_base, out_score, out_id, out_count, out_resolved, count_empty, out_redo, nullptr, stream);
}

int hq_refine_rescore_topk_pp(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                              const double* Zc, const double* Sc, int64_t N, int L, int mode,
                              const double* cand_score, const int64_t* cand_id, int kp, int k, double threshold,
                              int thr_mode, double eps, int64_t id_base, double* out_score, int64_t* out_id,
                              int* out_count, int* out_resolved, int count_empty, int* out_redo, int* next_redo,
                              double* out_det, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || kp <= 0 || kp > kMaxTopKBig || k <= 0 || k > kp)
    return fail(HQ_E_INVALID, "bad sizes kp=%d k=%d", kp, k);
  if (Q == 0) {  // no kernel runs: the next batch's counter is still cleared
    if (next_redo) HQ_CHECK_HIP(hipMemsetAsync(next_redo, 0, sizeof(int), (hipStream_t)stream));
    return HQ_OK;
  }
  if (!Rq || !Zq || !Sq || !cand_score || !cand_id || !out_score || !out_id || !out_count || !out_resolved ||
      !out_det || !out_redo || !next_redo || out_redo == next_redo || (N > 0 && (!Rc || !Zc || !Sc)))
    return fail(HQ_E_INVALID, "null buffer");
  return refine_launch(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps,
                       id_base, out_score, out_id, out_count, out_resolved, count_empty, out_redo, out_det, stream,
                       next_redo);
}

int hq_refine_rescore_topk(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                           const double* Zc, const double* Sc, int64_t N, int L, int mode, const double* cand_score,
                           const int64_t* cand_id, int kp, int k, double threshold, int thr_mode, double eps,
                           int64_t id_base, double* out_score, int64_t* out_id, int* out_count, int* out_resolved,
                           int count_empty, int* out_redo, double* out_det, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || kp <= 0 || kp > kMaxTopKBig || k <= 0 || k > kp)
    return fail(HQ_E_INVALID, "bad sizes kp=%d k=%d", kp, k);
  if (Q == 0) return HQ_OK;
  if (!Rq || !Zq || !Sq || !cand_score || !cand_id || !out_score || !out_id || !out_count || !out_resolved ||
      !out_det || (N > 0 && (!Rc || !Zc || !Sc)))
    return fail(HQ_E_INVALID, "null buffer");
  return refine_launch(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps,
                       id_base, out_score, out_id, out_count, out_resolved, count_empty, out_redo, out_det, stream);
}

size_t hq_refine_workspace_size(int Q, int kp, int L) { return refine_ws_bytes(Q, kp, L); }

int hq_refine_topk_ws(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc, const double* Zc,
                      const double* Sc, int64_t N, int L, int mode, const double* cand_score, const int64_t* cand_id,
                      int kp, int k, double threshold, int thr_mode, double eps, int64_t id_base, double* out_score,
                      int64_t* out_id, int* out_count, int* out_resolved, int count_empty, int* out_redo,
                      int* next_redo, double* out_det, void* workspace, size_t workspace_bytes, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || kp <= 0 || kp > kMaxTopKBig || k <= 0 || k > kp)
    return fail(HQ_E_INVALID, "bad sizes kp=%d k=%d", kp, k);
  if (Q == 0) {  // no kernel runs: the next batch's counter is still cleared
    if (next_redo) HQ_CHECK_HIP(hipMemsetAsync(next_redo, 0, sizeof(int), (hipStream_t)stream));
    return HQ_OK;
  }
  if (!Rq || !Zq || !Sq || !cand_score || !cand_id || !out_score || !out_id || !out_count || !out_resolved ||
      (next_redo && (!out_redo || out_redo == next_redo)) || (N > 0 && (!Rc || !Zc || !Sc)))
    return fail(HQ_E_INVALID, "null buffer");
  if (workspace && workspace_bytes < hq_refine_workspace_size(Q, kp, L)) return fail(HQ_E_INVALID, "workspace too small");
  return refine_launch(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps,
                       id_base, out_score, out_id, out_count, out_resolved, count_empty, out_redo, out_det, stream,
                       next_redo, workspace, workspace_bytes);
}

int hq_refine_final_ws(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc, const double* Zc,
                       const double* Sc, int64_t N, int L, const double* cand_score, const int64_t* cand_id, int kp,
                       int k, double threshold, int thr_mode, double eps, int64_t id_base, double* out_score,
                       int64_t* out_id, int* out_count, int* out_resolved, int* out_redo, int* next_redo, int K_out,
                       int64_t* fin_id, double* fin_det, int* fin_count, void* workspace, size_t workspace_bytes,
                       hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || kp <= 0 || kp > kMaxTopKBig || k <= 0 || k > kp || K_out <= 0)
    return fail(HQ_E_INVALID, "bad sizes kp=%d k=%d K=%d", kp, k, K_out);
  SegInfo si;
  seg_info(L, si);
  // the fused form exists on the lane-cooperative paths only (k_rank_small for lists <= 64, k_rank_pairs +
  // k_rank_sort above; the caller keeps the two-step form otherwise: hq_refine_topk_ws + hq_progressive_final_ex)
  const bool small = kp <= kMaxTopK && coop_ppl(si) && opt(OPT_REFINE_SMALL, 1) != 0;
  const bool big = kp > kMaxTopK && coop_ppl(si) && opt(OPT_REFINE_COOP, 1) != 0 && Q <= 65535;
  if (!small && !big) return fail(HQ_E_UNSUPPORTED, "fused final ranking: kp=%d L=%d", kp, L);
  if (Q == 0) {
    if (next_redo) HQ_CHECK_HIP(hipMemsetAsync(next_redo, 0, sizeof(int), (hipStream_t)stream));
    return HQ_OK;
  }
  // out_score / out_id may both be null: the level-0 lists are then not written
  if (!Rq || !Zq || !Sq || !cand_score || !cand_id || (!out_score != !out_id) || !out_count || !out_resolved ||
      !fin_id || !fin_det || !fin_count || (big && !workspace) || (next_redo && (!out_redo || out_redo == next_redo)) ||
      (N > 0 && (!Rc || !Zc || !Sc)))
    return fail(HQ_E_INVALID, "null buffer");
  if (big && workspace_bytes < hq_refine_workspace_size(Q, kp, L)) return fail(HQ_E_INVALID, "workspace too small");
  const FinalOut fin{K_out, fin_id, fin_det, fin_count, opt(OPT_FINAL_ROUNDS, 1) != 0 ? 1 : 0};
  // records on (the final ranking reads them from the workspace), count_empty on (nothing passed: redo)
  double* dummy_det = fin_det;
  return refine_launch(Rq, Zq, Sq, Q, Rc, Zc, Sc, N, L, 0, cand_score, cand_id, kp, k, threshold, thr_mode, eps,
                       id_base, out_score, out_id, out_count, out_resolved, 1, out_redo, dummy_det, stream, next_redo,
                       workspace, workspace_bytes, &fin);
}

size_t hq_scan_workspace_size(int Q, int64_t N, int k) {
  if (k > kMaxTopK) return scan0_ws_bytes(Q, N, k);  // long lists: the split level-0 scan only
  int nqb, nchunks;
  int64_t chunk_len;
  scan_geometry(Q, N, nqb, nchunks, chunk_len);
  const size_t w1 = (size_t)nchunks * Q * k * 16 + (size_t)nchunks * Q * 16 + 256;
  const size_t w0 = scan0_ws_bytes(Q, N, k);
  return w0 > w1 ? w0 : w1;
}

int hq_scan_topk(const double* Zq, const double* Sq, int Q, const double* Zc, const double* Sc, int64_t N, int L,
                 int mode, int k, double threshold, int thr_mode, int64_t id_base, void* workspace,
                 size_t workspace_bytes, double* out_score, int64_t* out_id, double* out_best,
                 int64_t* out_best_id, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (k <= 0 || k > kMaxTopK) return fail(HQ_E_UNSUPPORTED, "k=%d (1..%d)", k, kMaxTopK);
  if (mode != 0 && mode != 1) return fail(HQ_E_INVALID, "mode %d", mode);
  if (Q == 0) return HQ_OK;
  if (!out_score || !out_id) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (N == 0) {
    HQ_CHECK_HIP(hipMemsetAsync(out_id, 0xFF, sizeof(int64_t) * Q * k, s));
    if (out_best_id) HQ_CHECK_HIP(hipMemsetAsync(out_best_id, 0xFF, sizeof(int64_t) * Q, s));
    return HQ_OK;
  }
  if (!Zq || !Sq || !Zc || !Sc || !workspace) return fail(HQ_E_INVALID, "null buffer");
  if (workspace_bytes < hq_scan_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
#ifdef HQ_DIAG
  // diagnostics builds: the f64 wave-level level-0 scan (option scan_variant = 64)
  if (mode == 0 && !out_best && !out_best_id && N < 0x7FFFFFFF && opt(OPT_SCAN_VARIANT, 0) == 64) {
    SegInfo si;
    seg_info(L, si);
    const int ks = si.plen[0] / 4;
    if (ks >= 1 && ks <= 8)
      return scan0_run(false, ks, Zq, Sq, nullptr, nullptr, Q, Zc, Sc, nullptr, nullptr, N, si, k, threshold,
                       thr_mode, id_base, workspace, out_score, out_id, s);
  }
#endif
  ScanArgs a;
  a.Zq = Zq; a.Sq = Sq; a.Q = Q; a.Zc = Zc; a.Sc = Sc; a.N = N;
  seg_info(L, a.si);
  const int kp = mode == 0 ? a.si.plen[0] : a.si.Lp;
  a.ks = kp / 4;
  a.nseg_used = mode == 0 ? 1 : a.si.nseg;
  a.rs = rs_for(kp);
  a.K = k;
  a.thr = threshold;
  a.thr_mode = thr_mode;
  a.id_base = id_base;
  scan_geometry(Q, N, a.nqb, a.nchunks, a.chunk_len);
  uint8_t* ws = reinterpret_cast<uint8_t*>(workspace);
  a.ws_score = reinterpret_cast<double*>(ws);
  a.ws_id = reinterpret_cast<int64_t*>(ws + (size_t)a.nchunks * Q * k * 8);
  a.ws_best = reinterpret_cast<double*>(ws + (size_t)a.nchunks * Q * k * 16);
  a.ws_best_id = reinterpret_cast<int64_t*>(ws + (size_t)a.nchunks * Q * k * 16 + (size_t)a.nchunks * Q * 8);
  int rc;
  if (mode == 0) {
    if (a.ks <= 8) rc = launch_scan<8, false>(a, s);
    else if (a.ks <= 16) rc = launch_scan<16, false>(a, s);
    else if (a.ks <= 32) rc = launch_scan<32, false>(a, s);
    else if (a.ks <= 64) rc = launch_scan<64, false>(a, s);
    else return fail(HQ_E_UNSUPPORTED, "level-0 segment too long (%d)", kp);
  } else {
    if (a.ks <= 8) rc = launch_scan<8, true>(a, s);
    else if (a.ks <= 16) rc = launch_scan<16, true>(a, s);
    else if (a.ks <= 32) rc = launch_scan<32, true>(a, s);
    else if (a.ks <= 64) rc = launch_scan<64, true>(a, s);
    else return fail(HQ_E_UNSUPPORTED, "index too long for the fused scan (Lp=%d)", kp);
  }
  if (rc) return rc;
  int mg = Q < 4096 ? Q : 4096;
  hipLaunchKernelGGL(k_merge, dim3(mg), dim3(64), 0, s, a.ws_score, a.ws_id, a.ws_best, a.ws_best_id, a.nchunks, Q,
                     k, out_score, out_id, out_best, out_best_id);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_seg_level0_len(int L) {
  SegInfo si;
  seg_info(L, si);
  return si.nseg > 0 ? si.plen[0] : 0;
}

int hq_seg_prepare_pack0(const double* idx, int64_t N, int L, int src_f32, const uint8_t* row_f32, double* Z,
                         double* stats, void* Z16, float* S32, hq_stream_t stream) {
  if (L <= 0 || N < 0) return fail(HQ_E_INVALID, "bad shape N=%lld L=%d", (long long)N, L);
  if ((N > 0 && (!idx || !Z || !stats)) || !Z16 || !S32) return fail(HQ_E_INVALID, "null buffer");
  SegInfo si;
  seg_info(L, si);
  if (si.nseg == 0) return fail(HQ_E_INVALID, "no level structure for L=%d", L);
  if (si.plen[0] > 32) return fail(HQ_E_UNSUPPORTED, "level-0 segment of %d values (<= 32)", si.plen[0]);
  if (si.L > 4096) return fail(HQ_E_UNSUPPORTED, "L=%d (<= 4096)", L);
  const int64_t rows = z16_rows(N);
  // default: the lane-cooperative form where its shapes hold (option prep_coop = 0: the serial form)
  if (seg_small(si) && si.nseg <= 8 && opt(OPT_PREP_COOP, 1) != 0) {
    hipLaunchKernelGGL(k_seg_prepare_pack0_coop, dim3((unsigned)(rows < 65536 ? rows : 65536)), dim3(64),
                       (size_t)8 * si.L, (hipStream_t)stream, idx, N, si, src_f32 ? 1 : 0, row_f32, Z, stats,
                       reinterpret_cast<_Float16*>(Z16), S32);
    HQ_CHECK_LAUNCH();
    return HQ_OK;
  }
  hipLaunchKernelGGL(k_seg_prepare_pack0, dim3((unsigned)(rows < 65536 ? rows : 65536)), dim3(64), (size_t)8 * si.L,
                     (hipStream_t)stream, idx, N, si, src_f32 ? 1 : 0, row_f32, Z, stats,
                     reinterpret_cast<_Float16*>(Z16), S32);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_seg_pack0_split(const double* Z, const double* S, int64_t N, int L, void* Z16, float* S32,
                       hq_stream_t stream) {
  if (L <= 0 || N < 0) return fail(HQ_E_INVALID, "bad shape N=%lld L=%d", (long long)N, L);
  if ((N > 0 && (!Z || !S)) || !Z16 || !S32) return fail(HQ_E_INVALID, "null buffer");
  SegInfo si;
  seg_info(L, si);
  if (si.nseg == 0) return fail(HQ_E_INVALID, "no level structure for L=%d", L);
  if (si.plen[0] > 32) return fail(HQ_E_UNSUPPORTED, "level-0 segment of %d values (<= 32)", si.plen[0]);
  int64_t blocks = (z16_rows(N) * 32 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_pack0, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, Z, S, N, si.Lp, si.plen[0],
                     si.nseg, reinterpret_cast<_Float16*>(Z16), S32);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_seg_flag_rows(const float* S32, int64_t N, int* flags, hq_stream_t stream) {
  if (N < 0) return fail(HQ_E_INVALID, "bad shape N=%lld", (long long)N);
  if (!flags || (N > 0 && !S32)) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  HQ_CHECK_HIP(hipMemsetAsync(flags, 0, sizeof(int), s));
  if (N == 0) return HQ_OK;
  const int64_t fb = (N + 255) / 256;
  hipLaunchKernelGGL(k_flag_rows, dim3((unsigned)(fb < 4096 ? fb : 4096)), dim3(256), 0, s, S32, N, flags + 1, flags);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_scan0_topk_split(const void* Zq16, const float* Sq32, const double* Sq, int Q, const void* Zc16,
                        const float* Sc32, const double* Sc, int64_t N, int L, int k, double threshold, int thr_mode,
                        int64_t id_base, void* workspace, size_t workspace_bytes, double* out_score,
                        int64_t* out_id, hq_stream_t stream) {
  return hq_scan0_topk_split_fl(Zq16, Sq32, Sq, Q, Zc16, Sc32, Sc, N, L, k, threshold, thr_mode, id_base, workspace,
                                workspace_bytes, out_score, out_id, nullptr, stream);
}

int hq_scan0_topk_split_fl(const void* Zq16, const float* Sq32, const double* Sq, int Q, const void* Zc16,
                           const float* Sc32, const double* Sc, int64_t N, int L, int k, double threshold,
                           int thr_mode, int64_t id_base, void* workspace, size_t workspace_bytes, double* out_score,
                           int64_t* out_id, const int* corpus_flags, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (k <= 0 || k > kMaxTopKBig) return fail(HQ_E_UNSUPPORTED, "k=%d (1..%d)", k, kMaxTopKBig);
  if (Q == 0) return HQ_OK;
  if (!out_score || !out_id) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (N == 0) {
    HQ_CHECK_HIP(hipMemsetAsync(out_id, 0xFF, sizeof(int64_t) * Q * k, s));
    return HQ_OK;
  }
  if (N >= 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "N=%lld rows (int32 row ids)", (long long)N);
  if (!Zq16 || !Sq32 || !Sq || !Zc16 || !Sc32 || !Sc || !workspace) return fail(HQ_E_INVALID, "null buffer");
  if (workspace_bytes < hq_scan_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
  SegInfo si;
  seg_info(L, si);
  const int ks = si.nseg > 0 ? si.plen[0] / 4 : 0;
  if (ks < 1 || ks > 8) return fail(HQ_E_UNSUPPORTED, "level-0 segment of %d values (1..32)", si.plen[0]);
  return scan0_run(true, ks, nullptr, Sq, reinterpret_cast<const _Float16*>(Zq16), Sq32, Q, nullptr, Sc,
                   reinterpret_cast<const _Float16*>(Zc16), Sc32, N, si, k, threshold, thr_mode, id_base, workspace,
                   out_score, out_id, s, corpus_flags);
}

int hq_rescore(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc, const double* Zc,
               const double* Sc, int64_t N, int L, const int64_t* ids, int k, int64_t id_base, double* out,
               hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0 || k < 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || k == 0) return HQ_OK;
  if (!Rq || !Zq || !Sq || !ids || !out || (N > 0 && (!Rc || !Zc || !Sc))) return fail(HQ_E_INVALID, "null buffer");
  SegInfo si;
  seg_info(L, si);
  const int64_t total = (int64_t)Q * k;
  const int G = si.nseg <= 8 ? 8 : 16;
  int64_t blocks = (total * G + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  const bool sm = seg_small(si);
  if (G == 8 && sm)
    hipLaunchKernelGGL((k_rescore<8, true>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, VecSet{Rq, Zq, Sq},
                       Q, VecSet{Rc, Zc, Sc}, N, si, ids, k, id_base, out);
  else if (G == 8)
    hipLaunchKernelGGL((k_rescore<8, false>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, VecSet{Rq, Zq, Sq},
                       Q, VecSet{Rc, Zc, Sc}, N, si, ids, k, id_base, out);
  else if (sm)
    hipLaunchKernelGGL((k_rescore<16, true>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, VecSet{Rq, Zq, Sq},
                       Q, VecSet{Rc, Zc, Sc}, N, si, ids, k, id_base, out);
  else
    hipLaunchKernelGGL((k_rescore<16, false>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream,
                       VecSet{Rq, Zq, Sq}, Q, VecSet{Rc, Zc, Sc}, N, si, ids, k, id_base, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_progressive_final(int R, int Q, int M, int nseg, const double* s0, const int64_t* ids, const double* det,
                         const double* best, const int64_t* best_id, const double* best_det, int K,
                         int64_t* out_id, double* out_det, int* out_count, hq_stream_t stream) {
  return hq_progressive_final_ex(R, Q, M, nseg, s0, ids, det, best, best_id, best_det, K, out_id, out_det, out_count,
                                 0, stream);
}

int hq_progressive_final_ex(int R, int Q, int M, int nseg, const double* s0, const int64_t* ids, const double* det,
                            const double* best, const int64_t* best_id, const double* best_det, int K,
                            int64_t* out_id, double* out_det, int* out_count, int flags, hq_stream_t stream) {
  if (R <= 0 || R > 16 || Q < 0 || M <= 0 || M > kMaxTopKBig || K <= 0 || nseg < 0 || nseg >= kMaxSeg)
    return fail(HQ_E_INVALID, "bad sizes R=%d Q=%d M=%d K=%d", R, Q, M, K);
  if (Q == 0) return HQ_OK;
  if (!s0 || !ids || !det || !best || !best_id || !best_det || !out_id || !out_det || !out_count)
    return fail(HQ_E_INVALID, "null buffer");
  const int W = 1 + nseg;
  const int grid = Q < 8192 ? Q : 8192;
  if (M <= kMaxTopK)
    hipLaunchKernelGGL(k_progressive_final, dim3(grid), dim3(64), 0, (hipStream_t)stream, R, Q, M, W, s0, ids, det,
                       best, best_id, best_det, K, out_id, out_det, out_count, flags);
  else
    hipLaunchKernelGGL(k_progressive_final_big, dim3(grid), dim3(256), 0, (hipStream_t)stream, R, Q, M, W, s0, ids,
                       det, best, best_id, best_det, K, out_id, out_det, out_count,
                       (flags & 1) | (opt(OPT_FINAL_ROUNDS, 1) != 0 ? 0 : 2));  // option final_rounds = 0: sort only
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

// parts of the two-stage select: ~8192 entries each, <= 1024 per query
static void select_parts(int Q, int64_t N, int& P, int64_t& plen) {
  int64_t p = (N + 8191) / 8192;
  if (p > 1024) p = 1024;
  if (p < 1) p = 1;
  P = (int)p;
  plen = (N + P - 1) / P;
}

// the register-resident multi-stage select runs when the two-stage form would have few waves
static bool select_reg_ok(int Q, int64_t N, int k) {
  return N > 0 && k >= 16 && k <= 64 && (int64_t)Q * ((N + 8191) / 8192) < 4096 && !opt_on(OPT_SELECT_2STAGE);
}
static int64_t select_reg_parts(int64_t N) { return (N + kRegSel - 1) / kRegSel; }

// the sort-based select (k > 64): stage-1 parts of the row and their ping-pong stage buffers
static bool select_sort_ok(int64_t N, int k) {
  return N > 0 && k > kMaxTopK && k <= kSortPart / 4 && !opt_on(OPT_SELECT_2STAGE);
}
static int64_t select_sort_parts(int64_t N) { return (N + kSortPart - 1) / kSortPart; }

size_t hq_select_workspace_size(int Q, int64_t N, int k) {
  if (Q <= 0 || N <= 0 || k <= 0) return 0;
  if (select_sort_ok(N, k)) {  // two k-list stage buffers + the stage-1 arg-maxes
    const size_t P1 = (size_t)select_sort_parts(N);
    return 2 * (size_t)Q * P1 * k * 16 + (size_t)Q * P1 * 16 + 512;
  }
  int P;
  int64_t plen;
  select_parts(Q, N, P, plen);
  size_t two = (size_t)Q * P * ((size_t)k + 1) * 16 + 256;
  if (select_reg_ok(Q, N, k)) {  // two ping-pong stage buffers of the stage-1 size
    const size_t reg = 2 * (size_t)Q * select_reg_parts(N) * ((size_t)k + 1) * 16 + 256;
    if (reg > two) two = reg;
  }
  return two;
}

int hq_select_topk_ws(const double* scores, int Q, int64_t N, int k, double threshold, int thr_mode,
                      int64_t id_base, void* workspace, size_t workspace_bytes, double* out_score, int64_t* out_id,
                      double* out_best, int64_t* out_best_id, hq_stream_t stream) {
  if (Q < 0 || N < 0 || k <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0) return HQ_OK;
  if (workspace && out_score && out_id && scores && select_sort_ok(N, k)) {
    if (workspace_bytes < hq_select_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t P1 = select_sort_parts(N);
    const size_t cap = (size_t)Q * P1 * k;
    uint8_t* w = reinterpret_cast<uint8_t*>(workspace);
    double* bs[2] = {reinterpret_cast<double*>(w), reinterpret_cast<double*>(w + cap * 16)};
    int64_t* bi[2] = {reinterpret_cast<int64_t*>(w + cap * 8), reinterpret_cast<int64_t*>(w + cap * 24)};
    double* pb = reinterpret_cast<double*>(w + cap * 32);
    int64_t* pbi = reinterpret_cast<int64_t*>(w + cap * 32 + (size_t)Q * P1 * 8);
    // stage 1: parts of the row (the arg-maxes per part, or straight to the outputs when one part)
    const int64_t part1 = (N + P1 - 1) / P1;
    bool last = P1 == 1;
    int64_t g = (int64_t)Q * P1 < 65536 ? (int64_t)Q * P1 : 65536;
    hipLaunchKernelGGL(k_select_sort, dim3((unsigned)g), dim3(512), 0, s, scores, (const int64_t*)nullptr, Q, N, part1,
                       (int)P1, k, threshold, thr_mode, last ? 1 : 0, id_base, last ? out_score : bs[0],
                       last ? out_id : bi[0], last ? out_best : pb, last ? out_best_id : pbi, (const double*)nullptr,
                       (const int64_t*)nullptr, 0);
    HQ_CHECK_LAUNCH();
    int64_t P = P1;
    int cur = 0;
    const int64_t F = kSortPart / k;  // k-lists merged per part (>= 4)
    while (P > 1) {
      const int64_t P2 = (P + F - 1) / F;
      last = P2 == 1;
      g = (int64_t)Q * P2 < 65536 ? (int64_t)Q * P2 : 65536;
      hipLaunchKernelGGL(k_select_sort, dim3((unsigned)g), dim3(512), 0, s, (const double*)bs[cur],
                         (const int64_t*)bi[cur], Q, P * k, F * k, (int)P2, k, threshold, thr_mode, last ? 1 : 0,
                         id_base, last ? out_score : bs[cur ^ 1], last ? out_id : bi[cur ^ 1],
                         last ? out_best : (double*)nullptr, last ? out_best_id : (int64_t*)nullptr,
                         (const double*)pb, (const int64_t*)pbi, (int)P1);
      HQ_CHECK_LAUNCH();
      P = P2;
      cur ^= 1;
    }
    return HQ_OK;
  }
  int P;
  int64_t plen;
  select_parts(Q, N, P, plen);
  if (workspace && out_score && out_id && scores && select_reg_ok(Q, N, k) && P > 1) {
    if (workspace_bytes < hq_select_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t P1 = select_reg_parts(N);
    const int F = kRegSel / k < 64 ? kRegSel / k : 64;  // fan-in: F k <= kRegSel candidates, F <= 64 arg-maxes
    const size_t cap = (size_t)Q * P1;                   // parts a stage buffer holds
    uint8_t* w = reinterpret_cast<uint8_t*>(workspace);
    auto region = [&](int r, double*& rs, int64_t*& ri, double*& rb, int64_t*& rbi) {
      uint8_t* b = w + (size_t)r * cap * ((size_t)k + 1) * 16;
      rs = reinterpret_cast<double*>(b);
      ri = reinterpret_cast<int64_t*>(b + cap * k * 8);
      rb = reinterpret_cast<double*>(b + cap * k * 16);
      rbi = reinterpret_cast<int64_t*>(b + cap * k * 16 + cap * 8);
    };
    double *as, *bs_, *ab, *bb;
    int64_t *ai, *bi, *abi, *bbi;
    region(0, as, ai, ab, abi);
    region(1, bs_, bi, bb, bbi);
    // every stage keeps the arg-maxes (the final one writes them only when requested)
    int64_t P = P1;
    const bool last1 = P == 1;
    int64_t g = (int64_t)Q * P < 65536 ? (int64_t)Q * P : 65536;
    hipLaunchKernelGGL(k_select_reg1, dim3((unsigned)g), dim3(64), 0, s, scores, Q, N, (int)P, k, threshold, thr_mode,
                       last1 ? id_base : 0, last1 ? out_score : as, last1 ? out_id : ai, last1 ? out_best : ab,
                       last1 ? out_best_id : abi);
    HQ_CHECK_LAUNCH();
    int cur = 0;
    while (P > 1) {
      const int64_t P2 = (P + F - 1) / F;
      const bool last = P2 == 1;
      double *is_, *ib, *os_, *ob;
      int64_t *ii, *ibi, *oi, *obi;
      if (cur == 0) { is_ = as; ii = ai; ib = ab; ibi = abi; os_ = bs_; oi = bi; ob = bb; obi = bbi; }
      else { is_ = bs_; ii = bi; ib = bb; ibi = bbi; os_ = as; oi = ai; ob = ab; obi = abi; }
      g = (int64_t)Q * P2 < 65536 ? (int64_t)Q * P2 : 65536;
      hipLaunchKernelGGL(k_select_regm, dim3((unsigned)g), dim3(64), 0, s, Q, (int)P, F, (int)P2, k,
                         last ? id_base : 0, (const double*)is_, (const int64_t*)ii, (const double*)ib,
                         (const int64_t*)ibi, last ? out_score : os_, last ? out_id : oi, last ? out_best : ob,
                         last ? out_best_id : obi);
      HQ_CHECK_LAUNCH();
      P = P2;
      cur ^= 1;
    }
    return HQ_OK;
  }
  if (P == 1 || !workspace)
    return hq_select_topk(scores, Q, N, k, threshold, thr_mode, id_base, out_score, out_id, out_best, out_best_id,
                          stream);
  if (!out_score || !out_id || !scores) return fail(HQ_E_INVALID, "null buffer");
  if (workspace_bytes < hq_select_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
  uint8_t* ws = reinterpret_cast<uint8_t*>(workspace);
  const size_t nk = (size_t)Q * P * k;
  double* ws_s = reinterpret_cast<double*>(ws);
  int64_t* ws_id = reinterpret_cast<int64_t*>(ws + nk * 8);
  double* ws_b = reinterpret_cast<double*>(ws + nk * 16);
  int64_t* ws_bid = reinterpret_cast<int64_t*>(ws + nk * 16 + (size_t)Q * P * 8);
  const int64_t g1 = (int64_t)Q * P < 65536 ? (int64_t)Q * P : 65536;
  hipLaunchKernelGGL(k_select_part, dim3((unsigned)g1), dim3(64), 0, (hipStream_t)stream, scores, Q, N, P, plen, k,
                     threshold, thr_mode, ws_s, ws_id, ws_b, ws_bid);
  HQ_CHECK_LAUNCH();
  const int g2 = Q < 4096 ? Q : 4096;
  hipLaunchKernelGGL(k_select_merge, dim3(g2), dim3(64), 0, (hipStream_t)stream, Q, P, k, threshold, thr_mode, id_base,
                     (const double*)ws_s, (const int64_t*)ws_id, (const double*)ws_b, (const int64_t*)ws_bid,
                     out_score, out_id, out_best, out_best_id);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_select_topk(const double* scores, int Q, int64_t N, int k, double threshold, int thr_mode, int64_t id_base,
                   double* out_score, int64_t* out_id, double* out_best, int64_t* out_best_id, hq_stream_t stream) {
  if (Q < 0 || N < 0 || k <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0) return HQ_OK;
  if (!out_score || !out_id || (N > 0 && !scores)) return fail(HQ_E_INVALID, "null buffer");
  int grid = Q < 4096 ? Q : 4096;
  hipLaunchKernelGGL(k_select, dim3(grid), dim3(64), 0, (hipStream_t)stream, scores, Q, N, k, threshold, thr_mode,
                     id_base, out_score, out_id, out_best, out_best_id);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_pair_scores_raw(const double* q, const double* C, int64_t N, int m, double* out, hq_stream_t stream) {
  return hq_pair_scores_raw_src(q, C, N, m, 0, 0, out, stream);
}

int hq_pair_scores_raw_src(const double* q, const double* C, int64_t N, int m, int q_f32, int c_f32, double* out,
                           hq_stream_t stream) {
  if (N < 0 || m <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (N == 0) return HQ_OK;
  if (!q || !C || !out) return fail(HQ_E_INVALID, "null buffer");
  int64_t blocks = (N + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_pair_raw, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, q, C, N, m, q_f32 ? 1 : 0,
                     c_f32 ? 1 : 0, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_cosine_scores(const float* a, int Q, const float* b, int64_t N, int K, double* out, hq_stream_t stream) {
  if (Q < 0 || N < 0 || K < 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || N == 0) return HQ_OK;
  if (!a || !b || !out) return fail(HQ_E_INVALID, "null buffer");
  const int64_t total = (int64_t)Q * N;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_cosine, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, a, Q, b, N, K, out);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}


/* ---- overall-mode scan (split-f16 copies of every level segment) ------------------------------ */
int hq_seg_packov_info(int L, int* nkb, int* ng, int* nc, int* group_floats) {
  OvLayout o;
  if (L <= 0 || !ov_layout(L, o)) return fail(HQ_E_UNSUPPORTED, "no split overall layout for L=%d", L);
  if (nkb) *nkb = o.nkb;
  if (ng) *ng = o.ng;
  if (nc) *nc = o.nc;
  if (group_floats) *group_floats = ov_gsize(o.ng, o.nc);
  return HQ_OK;
}

int hq_seg_packov_split(const double* Z, const double* S, int64_t N, int L, void* Zo16, float* So32,
                        hq_stream_t stream) {
  if (L <= 0 || N < 0) return fail(HQ_E_INVALID, "bad shape N=%lld L=%d", (long long)N, L);
  if ((N > 0 && (!Z || !S)) || !Zo16 || !So32) return fail(HQ_E_INVALID, "null buffer");
  if (N >= 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "N=%lld rows (int32 row ids)", (long long)N);
  OvLayout o;
  if (!ov_layout(L, o)) return fail(HQ_E_UNSUPPORTED, "no split overall layout for L=%d", L);
  SegInfo si;
  seg_info(L, si);
  int64_t blocks = (z16_rows(N) * o.nkb * 32 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_packov, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, Z, S, N, si.Lp, o,
                     reinterpret_cast<_Float16*>(Zo16), So32);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

size_t hq_scanov_workspace_size(int Q, int64_t N, int k) {
  if (Q <= 0 || N <= 0 || k <= 0) return 256;
  return ov_plan(Q, N, k).total;
}

int hq_scanov_topk_split(const void* Zq16, const float* Sq32, const double* Sq, const double* Zq, int Q,
                         const void* Zc16, const float* Sc32, const double* Sc, const double* Zc, int64_t N, int L,
                         int k, double threshold, int thr_mode, int64_t id_base, void* workspace,
                         size_t workspace_bytes, double* out_score, int64_t* out_id, hq_stream_t stream) {
  if (Q < 0 || N < 0 || L <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (k <= 0 || k > kMaxTopKBig) return fail(HQ_E_UNSUPPORTED, "k=%d (1..%d)", k, kMaxTopKBig);
  if (Q == 0) return HQ_OK;
  if (!out_score || !out_id) return fail(HQ_E_INVALID, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (N == 0) {
    HQ_CHECK_HIP(hipMemsetAsync(out_id, 0xFF, sizeof(int64_t) * Q * k, s));
    return HQ_OK;
  }
  if (N >= 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "N=%lld rows (int32 row ids)", (long long)N);
  if (!Zq16 || !Sq32 || !Sq || !Zq || !Zc16 || !Sc32 || !Sc || !Zc || !workspace) return fail(HQ_E_INVALID, "null buffer");
  if (workspace_bytes < hq_scanov_workspace_size(Q, N, k)) return fail(HQ_E_INVALID, "workspace too small");
  OvArgs a;
  if (!ov_layout(L, a.o)) return fail(HQ_E_UNSUPPORTED, "no split overall layout for L=%d", L);
  SegInfo si;
  seg_info(L, si);
  const OvPlan p = ov_plan(Q, N, k);
  a.Zq = reinterpret_cast<const _Float16*>(Zq16); a.Sq32 = Sq32; a.Sq = Sq; a.Q = Q;
  a.Zc = reinterpret_cast<const _Float16*>(Zc16); a.Sc32 = Sc32; a.Sc = Sc; a.N = N;
  a.Zq64 = Zq; a.Zc64 = Zc; a.Lp = si.Lp;
  a.nqb = p.nqb; a.nchunks = p.nchunks; a.chunk_len = p.chunk_len;
  a.stride = p.stride; a.S = p.S; a.top = nullptr; a.qc = nullptr;
  const int sample_kth = scan_kprime(k, p.stride);
  const double thr0 = thr_mode == 0 ? -__builtin_huge_val() : threshold;
  uint8_t* ws = reinterpret_cast<uint8_t*>(workspace);
  if (a.o.lid == 0) return ov_launch<0>(a, p, si, k, thr0, sample_kth, id_base, ws, out_score, out_id, s);
  return ov_launch<1>(a, p, si, k, thr0, sample_kth, id_base, ws, out_score, out_id, s);
}

}  // extern "C"
