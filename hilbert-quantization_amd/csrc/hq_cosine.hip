// hq_cosine.hip — dense frame similarity on the matrix cores (north star: "the
// frame similarity as a batched L2/dot over N x (side x side) images — MFMA for the dense
// query x corpus contraction").
//
// Reference: rag/search/engine.py:622-660 _calculate_embedding_cosine_similarity — flatten, truncate
// to the common length, dot / (|a| |b|), (cos + 1) / 2, 0.0 when a norm is 0 — applied to every
// (query, stored frame) pair by the RAG search loops (:503-507, :1025-1051).  The reference computes
// in float32 through BLAS (sdot / snrm2 order), so scores agree within the north star's 1e-5, not bit
// for bit (DESIGN.md §4.5 has the error budget).
//
// Layout (hq_cos_prepare, once per corpus / query batch): every row x is scaled by a power of two s
// (max |s x| in [0.5, 1)) and split as hi = f16(s x), lo = f16(s x - hi), Kp = K rounded up to 32, stored
// as 1 KiB MFMA operand fragments (16-row tile, K step of 32, plane hi / lo: see cos_frag), plus inv[row] =
// 1 / (s |x|) (f64 norm of the original values; 0 for a zero row).  dot(a, b) = (hi_a.hi_b + hi_a.lo_b +
// lo_a.hi_b) / (s_a s_b) + O(2^-22 |a||b|).
//
// GEMM (default k_cos_t<3, 1, 1>): workgroup = 8 waves, tile 128 queries x 384 frames, wave w = all 128
// queries x frames 48 w .. + 47 (8 x 3 tiles of v_mfma_f32_16x16x32_f16 x 3: hi.hi, hi.lo, lo.hi), K steps
// of 32.  Query fragments go through LDS (register-staged, two stages, read by every wave); frame
// fragments, each used by one wave only, go straight from global memory into that wave's VGPRs one K step
// ahead.  Ping-pong: the two waves of every SIMD run one barrier phase apart (memory phase / 72 MFMAs).
// XCD-aware block order: the query tiles of one frame tile run back to back on one XCD, so the frame tile
// is read from HBM once.  Epilogue: (acc * inv_q * inv_c + 1) / 2, f64 stores.  A/B forms (option
// cos_kernel): the LDS-DMA kernel k_cos_g3 (ping-pong / lockstep) and the register-staged
// k_cos_mfma on the row-major layout, and other k_cos_t tiles / prefetch distances / epilogues.
#include "hq_common.h"

#include <stdlib.h>
#include <string.h>

namespace hq {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

constexpr int kCosT = 128;                 // tile rows (queries) = tile cols (frames)
constexpr int kCosK = 32;                  // K per step
constexpr int kCosRow = 40;                // LDS halves per tile row (32 + 8 pad: 80 B)

// ---- prepare: scale, split, inverse norm ------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cos_prepare(const float* __restrict__ X, int64_t N, int64_t ld, int K,
                                                     int Kp, int64_t rows_out, _Float16* __restrict__ X16,
                                                     double* __restrict__ inv) {
  // one wave per row
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = w0; r < rows_out; r += nw) {
    _Float16* hi = X16 + r * 2 * Kp;
    _Float16* lo = hi + Kp;
    if (r >= N) {  // pad rows: zeros, inv 0
      for (int k = lane; k < Kp; k += 64) hi[k] = lo[k] = (_Float16)0.0f;
      if (lane == 0) inv[r] = 0.0;
      continue;
    }
    const float* x = X + r * ld;
    float amax = 0.0f;
    double ss = 0.0;
    for (int k = lane; k < K; k += 64) {
      const float v = x[k];
      amax = fmaxf(amax, fabsf(v));
      ss = fma((double)v, (double)v, ss);
    }
    for (int o = 32; o > 0; o >>= 1) {
      amax = fmaxf(amax, __shfl_xor(amax, o, 64));
      ss += __shfl_xor(ss, o, 64);
    }
    int e = 0;
    if (amax > 0.0f) frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1)
    const float s = ldexpf(1.0f, -e);   // s x in (-1, 1)
    for (int k = lane; k < Kp; k += 64) {
      const float v = k < K ? x[k] * s : 0.0f;
      const _Float16 h = (_Float16)v;
      hi[k] = h;
      lo[k] = (_Float16)(v - (float)h);
    }
    if (lane == 0) inv[r] = ss > 0.0 ? 1.0 / ((double)s * sqrt(ss)) : 0.0;
  }
}

// ---- tiled fragment layout (default) ------------------------------------------------------------------
// Fragment (16-row tile t, K step kb, plane p) = 512 halves (1 KiB) at ((t KB + kb) 2 + p) 512, KB = Kp / 32;
// lane 16 g + j holds row 16 t + j, k = 32 kb + 8 g .. + 7 — exactly the v_mfma_f32_16x16x32_f16 A / B
// operand, so one fragment is one contiguous 1 KiB wave load (16 B per lane) and, staged in LDS
// lane-linearly, one bank-conflict-free ds_read_b128.
__device__ __forceinline__ int64_t cos_frag(int64_t t, int kb, int KB, int p) {
  return ((t * KB + kb) * 2 + p) * 512;
}

__global__ __launch_bounds__(1024) void k_cos_prepare_tiled(const float* __restrict__ X, int64_t N, int64_t ld, int K,
                                                            int Kp, int64_t rows_out, _Float16* __restrict__ X16,
                                                            double* __restrict__ inv) {
  // one 16-wave workgroup per 16-row tile: wave w takes row w's statistics in k_cos_prepare's lane-strided
  // order (same scale and inverse-norm bits), then the waves split the tile's K steps; per K step lane
  // 16 g + j converts row j's values 8 g .. 8 g + 7, so every fragment leaves as one contiguous 1 KiB wave
  // store per plane
  __shared__ float sc[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, j = lane & 15, g = lane >> 4;
  const int KB = Kp / kCosK;
  // blockIdx.y: one of gridDim.y parts of the K steps (small batches: more workgroups per tile, each
  // recomputing the tile's statistics)
  const int per = (KB + gridDim.y - 1) / gridDim.y;
  const int kb0 = blockIdx.y * per, kb1 = kb0 + per < KB ? kb0 + per : KB;
  for (int64_t t = blockIdx.x; t < rows_out / 16; t += gridDim.x) {
    const int64_t r0 = 16 * t + wv;
    if (r0 >= N) {  // pad rows: zeros (scale 0), inv 0
      if (lane == 0) {
        sc[wv] = 0.0f;
        if (blockIdx.y == 0) inv[r0] = 0.0;
      }
    } else {
      const float* x = X + r0 * ld;
      float amax = 0.0f;
      double ss = 0.0;
      for (int k = lane; k < K; k += 64) {
        const float v = x[k];
        amax = fmaxf(amax, fabsf(v));
        ss = fma((double)v, (double)v, ss);
      }
      for (int o = 32; o > 0; o >>= 1) {
        amax = fmaxf(amax, __shfl_xor(amax, o, 64));
        ss += __shfl_xor(ss, o, 64);
      }
      int e = 0;
      if (amax > 0.0f) frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1)
      const float s = ldexpf(1.0f, -e);   // s x in (-1, 1)
      if (lane == 0) {
        sc[wv] = s;
        if (blockIdx.y == 0) inv[r0] = ss > 0.0 ? 1.0 / ((double)s * sqrt(ss)) : 0.0;
      }
    }
    __syncthreads();
    const int64_t r = 16 * t + j;
    const float my_s = sc[j];
    const float* x = X + (r < N ? r : 0) * ld;
    for (int kb = kb0 + wv; kb < kb1; kb += 16) {
      h8 hi, lo;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = kCosK * kb + 8 * g + u;
        const float v = (r < N && k < K) ? x[k] * my_s : 0.0f;
        const _Float16 h = (_Float16)v;
        hi[u] = h;
        lo[u] = (_Float16)(v - (float)h);
      }
      _Float16* f = X16 + cos_frag(t, kb, KB, 0) + 8 * lane;
      *reinterpret_cast<h8*>(f) = hi;
      *reinterpret_cast<h8*>(f + 512) = lo;
    }
    __syncthreads();  // sc is rewritten by the next tile
  }
}

// ---- GEMM + epilogue ---------------------------------------------------------------------------------
struct CosArgs {
  const _Float16* A;  // queries [Qp, 2, Kp]
  const _Float16* B;  // frames  [Np, 2, Kp]
  const double* ia;   // [Qp]
  const double* ib;   // [Np]
  int Q;
  int64_t N;
  int Kp;
  int qtiles;
  int64_t ntiles;
  double* out;  // [Q, N]
  float* outf;  // [Q, N] float32 scores (hq_cos_scores_mfma_f32; k_cos_t EP 3): the reference's precision
};

// Register-staged baseline.  TQ = query rows per workgroup tile; frames per tile kCosT = 128.  LDS per
// buffer: (2 TQ + 2 * 128) rows of 80 B.
template <int TQ>
__global__ __launch_bounds__(256) void k_cos_mfma(CosArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cos_smem[];
  constexpr int kBuf = (2 * TQ + 2 * kCosT) * kCosRow;  // halves per buffer
  _Float16* lds0 = reinterpret_cast<_Float16*>(cos_smem);
  // plane p of buffer b: A hi / A lo (TQ rows), B hi / B lo (128 rows)
  auto plane = [&](int b, int p) -> _Float16* {
    return lds0 + b * kBuf + (p < 2 ? p * TQ * kCosRow : 2 * TQ * kCosRow + (p - 2) * kCosT * kCosRow);
  };
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // XCD-aware order: blocks with equal (blockIdx % 8) share an XCD; the query tiles of a frame tile
  // are consecutive within one XCD's sequence
  const int64_t blk = blockIdx.x;
  const int64_t xcd = blk & 7, slot = blk >> 3;
  const int qt = (int)(slot % a.qtiles);
  const int64_t nt = xcd + 8 * (slot / a.qtiles);
  if (nt >= a.ntiles) return;
  const int64_t q0 = (int64_t)qt * TQ, n0 = nt * kCosT;
  const int Kp = a.Kp;
  // global -> register staging: A planes TQ rows, B planes 128 rows, 4 chunks of 16 B per row
  constexpr int CA = TQ * 4 / 256, CB = kCosT * 4 / 256;  // chunks per thread per plane
  h8 sa[2][CA], sb[2][CB];
  auto load_step = [&](int k0) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + 256 * i, row = c >> 2, seg = c & 3;
        sa[p][i] = *reinterpret_cast<const h8*>(a.A + ((q0 + row) * 2 + p) * (int64_t)Kp + k0 + 8 * seg);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + 256 * i, row = c >> 2, seg = c & 3;
        sb[p][i] = *reinterpret_cast<const h8*>(a.B + ((n0 + row) * 2 + p) * (int64_t)Kp + k0 + 8 * seg);
      }
    }
  };
  auto store_step = [&](int buf) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + 256 * i, row = c >> 2, seg = c & 3;
        *reinterpret_cast<h8*>(plane(buf, p) + row * kCosRow + 8 * seg) = sa[p][i];
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + 256 * i, row = c >> 2, seg = c & 3;
        *reinterpret_cast<h8*>(plane(buf, 2 + p) + row * kCosRow + 8 * seg) = sb[p][i];
      }
    }
  };
  // wave tile: queries (TQ/2) * (wv >> 1) .. + TQ/2, frames 64 * (wv & 1) .. +64
  constexpr int MI = TQ / 32;  // 16-row query tiles per wave
  const int wr = (TQ / 2) * (wv >> 1), wc = 64 * (wv & 1);
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  f4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int steps = Kp / kCosK;
  load_step(0);
  store_step(0);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int buf = s & 1;
    if (s + 1 < steps) load_step((s + 1) * kCosK);
    h8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = *reinterpret_cast<const h8*>(plane(buf, 2) + (wc + 16 * j + fr) * kCosRow + fk);
      bl[j] = *reinterpret_cast<const h8*>(plane(buf, 3) + (wc + 16 * j + fr) * kCosRow + fk);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const h8 ah = *reinterpret_cast<const h8*>(plane(buf, 0) + (wr + 16 * i + fr) * kCosRow + fk);
      const h8 al = *reinterpret_cast<const h8*>(plane(buf, 1) + (wr + 16 * i + fr) * kCosRow + fk);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // D[query row][frame col]: A operand = queries, B operand = frames, so each output row's 16
        // frames are 16 consecutive lanes (128-byte stores)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
      }
    }
    if (s + 1 < steps) store_step(buf ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds queries 4 (lane >> 4) + r of each 16-query tile, frame lane & 15
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t q = q0 + wr + 16 * i + 4 * (lane >> 4) + r;
      if (q >= a.Q) continue;
      const double iq = a.ia[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wc + 16 * j + fr;
        if (n >= a.N) continue;
        const double ic = a.ib[n];
        const double cs = (double)acc[i][j][r] * iq * ic;
        a.out[q * a.N + n] = (iq != 0.0 && ic != 0.0) ? (cs + 1.0) / 2.0 : 0.0;
      }
    }
}

// LDS-DMA staging: global_load_lds_dwordx4 writes each staged tile straight into LDS (no staging VGPRs,
// no ds_write).  The DMA destination is lane-linear (one wave instruction = 1 KiB = 16 rows of 64 B),
// so rows are unpadded and the bank spread comes from an XOR swizzle of the 16-byte segment applied
// on the SOURCE address and undone on the fragment read: physical seg = logical seg ^ kSw[(row >> 2) & 3].
// kSw = {0, 2, 3, 1} puts the sixteen rows of every ds_read_b128 lane group (lanes {0-3, 12-15,
// 20-27}, ... — MI355X_MICROARCH.md §LDS) on sixteen distinct 4-bank groups.
__device__ __forceinline__ int cos_sw(int g) { return (0x78 >> (2 * g)) & 3; }  // {0, 2, 3, 1}

// Three-stage LDS-DMA pipeline: tile 128 queries x TN frames, TN / 32 waves (each 64 x 64), K steps of
// 32, three LDS stages so the DMA of step s + 2 is in flight while step s computes (two steps of MFMA
// cover the HBM latency of the streamed frame rows).  The DMAs are inline asm (hipcc would otherwise
// drain them with vmcnt(0) at every barrier); each wave retires its own pieces of a stage with a
// counted vmcnt (the PW pieces of the next stage stay in flight) and an s_barrier publishes it.
// PP = 0: all waves in lockstep, one barrier per K step; PP = 1: ping-pong (below).
template <int TN, int PP, bool NTS = true>
__global__ __launch_bounds__(TN * 2) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_cos_g3(CosArgs a, int64_t np_rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cos_smem[];
  constexpr int TQ = 128, NW = TN / 32, kRow = kCosK, ST = 3;
  constexpr int kBuf = (2 * TQ + 2 * TN) * kRow;  // halves per stage
  constexpr int SA = TQ / 16, SB = TN / 16, NP = 2 * SA + 2 * SB, PW = NP / NW;
  static_assert(NP % NW == 0 && PW < 16, "pieces per wave");
  _Float16* lds0 = reinterpret_cast<_Float16*>(cos_smem);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t blk = blockIdx.x;
  const int64_t xcd = blk & 7, slot = blk >> 3;
  const int qt = (int)(slot % a.qtiles);
  const int64_t nt = xcd + 8 * (slot / a.qtiles);
  if (nt >= a.ntiles) return;
  const int64_t q0 = (int64_t)qt * TQ, n0 = nt * TN;
  const int Kp = a.Kp;
  const int lrow = lane >> 2;
  const int lseg = (lane & 3) ^ cos_sw((lane >> 4) & 3);
  const _Float16* src[PW];
  uint32_t dst[PW];  // LDS byte address of the piece in stage 0
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds0;
#pragma unroll
  for (int t = 0; t < PW; ++t) {
    const int i = wv + NW * t;
    int p, slab;
    if (i < 2 * SA) { p = i / SA; slab = i % SA; }
    else { p = 2 + (i - 2 * SA) / SB; slab = (i - 2 * SA) % SB; }
    const int64_t row = (int64_t)slab * 16 + lrow;
    const _Float16* base;
    if (p < 2) base = a.A + ((q0 + row) * 2 + p) * (int64_t)Kp;
    else {
      const int64_t rg = n0 + row < np_rows ? n0 + row : np_rows - 1;  // last tile may pass the padded rows
      base = a.B + (rg * 2 + (p - 2)) * (int64_t)Kp;
    }
    src[t] = base + 8 * lseg;
    const int off = (p < 2 ? p * TQ * kRow : 2 * TQ * kRow + (p - 2) * TN * kRow) + slab * 16 * kRow;
    dst[t] = __builtin_amdgcn_readfirstlane(lbase + 2 * off);
  }
  auto piece = [&](int t, int k0, int stage) {
    uint32_t keep;
    const _Float16* g = src[t] + k0;
    const uint32_t d = dst[t] + stage * (2 * kBuf);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(d) : "memory");
  };
  auto issue = [&](int k0, int stage) {
#pragma unroll
    for (int t = 0; t < PW; ++t) piece(t, k0, stage);
  };
  const int wr = 64 * (wv & 1), wc = 64 * (wv >> 1);
  const int fr = lane & 15;
  const int rseg = 8 * ((lane >> 4) ^ cos_sw(fr >> 2));
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int steps = Kp / kCosK;
  issue(0, 0);
  if (steps > 1) issue(kCosK, 1);
  int stage = 0;
  if constexpr (PP) {
    // Ping-pong: waves w and w + 4 share a SIMD; group 1 (waves 4-7) runs one barrier phase behind
    // group 0, so on every SIMD one wave issues its fragment reads + DMA while the other runs MFMAs.
    // Phases per K step: memory (DMA of step s + 2, 16 ds_read_b128, lgkmcnt(0)) then compute (48
    // MFMA), each closed by one block barrier.  Stage s + 1 is published at barrier 2s + 2: group 0
    // reaches it after computing step s, group 1 after its memory phase of step s; both retire it
    // with vmcnt(PW) (only the just-issued stage s + 2 stays in flight).  The lgkmcnt(0) before each
    // memory-phase barrier retires the reads of a stage before the other group's DMA may overwrite it.
    const int grp = __builtin_amdgcn_readfirstlane(wv >> 2);
    if (steps > 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (grp) asm volatile("s_barrier" ::: "memory");
    for (int s = 0; s < steps; ++s) {
      if (s + 2 < steps) issue((s + 2) * kCosK, stage == 0 ? 2 : stage - 1);
      const _Float16* pA = lds0 + stage * kBuf;
      const _Float16* pB = pA + 2 * TQ * kRow;
      h8 bh[4], bl[4], ah[4], al[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bh[j] = *reinterpret_cast<const h8*>(pB + (wc + 16 * j + fr) * kRow + rseg);
        bl[j] = *reinterpret_cast<const h8*>(pB + TN * kRow + (wc + 16 * j + fr) * kRow + rseg);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ah[i] = *reinterpret_cast<const h8*>(pA + (wr + 16 * i + fr) * kRow + rseg);
        al[i] = *reinterpret_cast<const h8*>(pA + TQ * kRow + (wr + 16 * i + fr) * kRow + rseg);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (grp) {
        if (s + 2 < steps) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (!grp) {
        if (s + 2 < steps) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        asm volatile("s_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      stage = stage == ST - 1 ? 0 : stage + 1;
    }
    if (!grp) asm volatile("s_barrier" ::: "memory");  // group 1's extra barrier: equal counts per wave
  } else
  for (int s = 0; s < steps; ++s) {
    // retire this wave's pieces of stage s (those of s + 1 may stay in flight), then publish
    if (s + 1 < steps) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + 2 < steps) issue((s + 2) * kCosK, stage == 0 ? 2 : stage - 1);
    const _Float16* pl = lds0 + stage * kBuf;
    const _Float16* pA = pl;
    const _Float16* pB = pl + 2 * TQ * kRow;
    // all sixteen fragments first (A rows 0-1 and B, then A rows 2-3 behind the first MFMAs); the
    // scheduling barriers keep the compiler from re-serialising the reads against the MFMAs
    h8 bh[4], bl[4], ah[4], al[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = *reinterpret_cast<const h8*>(pB + (wc + 16 * j + fr) * kRow + rseg);
      bl[j] = *reinterpret_cast<const h8*>(pB + TN * kRow + (wc + 16 * j + fr) * kRow + rseg);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = *reinterpret_cast<const h8*>(pA + (wr + 16 * i + fr) * kRow + rseg);
      al[i] = *reinterpret_cast<const h8*>(pA + TQ * kRow + (wr + 16 * i + fr) * kRow + rseg);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    stage = stage == ST - 1 ? 0 : stage + 1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t q = q0 + wr + 16 * i + 4 * (lane >> 4) + r;
      if (q >= a.Q) continue;
      const double iq = a.ia[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wc + 16 * j + fr;
        if (n >= a.N) continue;
        const double ic = a.ib[n];
        const double cs = (double)acc[i][j][r] * iq * ic;
        const double v = (iq != 0.0 && ic != 0.0) ? (cs + 1.0) / 2.0 : 0.0;
        if constexpr (NTS) __builtin_nontemporal_store(v, a.out + q * a.N + n);  // write-once scores
        else a.out[q * a.N + n] = v;
      }
    }
}

// Tiled-layout kernel (default).  Workgroup = 8 waves (2 per SIMD), tile 128 queries x 128 FT frames; wave
// w owns frames 16 FT w .. + 16 FT - 1 against all 128 queries (8 x FT accumulator tiles).  Only the query
// operand goes through LDS (16 fragments = 16 KiB per K step, two stages, register-staged: each wave loads
// and stores two of them), read by all 8 waves; every frame fragment is used by exactly one wave of the
// workgroup, so it goes straight from global memory into that wave's VGPRs (contiguous 1 KiB loads, two
// K steps ahead) and never touches LDS.  Per K step and wave: 16 ds_read_b128 + 2 ds_write_b128, 2 + 2 FT
// global loads, 24 FT MFMAs; one block barrier.  Per output the MFMA sequence is k_cos_g3's (per K step
// hi.hi, hi.lo, lo.hi), so the scores are bit-identical to it.
// X: diagnostics only (wrong scores; make DIAG=1): 1 no MFMAs, 2 no barriers in the K loop, 3 no frame
// loads after the prologue, 4 no query staging after the prologue, 5 no query fragment reads
template <int FT, int PP, int D, int EP, int X = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_cos_t(CosArgs a, int64_t ftiles) {
  // two query stages (32 KiB); after the K loop the epilogue stages one 16-query row block per wave here
  constexpr int kSm = 2 * 16 * 512 * 2 > 8 * 16 * 16 * FT * 8 ? 2 * 16 * 512 * 2 : 8 * 16 * 16 * FT * 8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kSm];
  _Float16(*sA)[16 * 512] = reinterpret_cast<_Float16(*)[16 * 512]>(smem);
  constexpr int QT = 8, TN = 8 * 16 * FT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t blk = blockIdx.x;
  const int64_t xcd = blk & 7, slot = blk >> 3;
  const int qt = (int)(slot % a.qtiles);
  const int64_t nt = xcd + 8 * (slot / a.qtiles);
  if (nt >= a.ntiles) return;
  const int KB = a.Kp / kCosK;
  const int64_t qt0 = (int64_t)qt * QT;
  // this thread's two query pieces per step: fragment f = wv + 8 i -> query tile f >> 1, plane f & 1
  const _Float16* srcA[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int f = wv + 8 * i;
    srcA[i] = a.A + cos_frag(qt0 + (f >> 1), 0, KB, f & 1) + 8 * lane;
  }
  const _Float16* srcB[FT];
#pragma unroll
  for (int j = 0; j < FT; ++j) {
    int64_t t = nt * (TN / 16) + wv * FT + j;
    if (t > ftiles - 1) t = ftiles - 1;  // the last frame tile may pass the padded rows
    srcB[j] = a.B + cos_frag(t, 0, KB, 0) + 8 * lane;
  }
  h8 ra[2];
  h8 rb0[FT][2], rb1[FT][2], rb2[FT][2];  // frame fragments of steps s, s + 1, s + 2 (a ring, unrolled by 3)
  auto loadA = [&](int kb) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = *reinterpret_cast<const h8*>(srcA[i] + (int64_t)kb * 1024);
  };
  auto loadB = [&](int kb, h8 (&d)[FT][2]) {
#pragma unroll
    for (int j = 0; j < FT; ++j) {
      d[j][0] = *reinterpret_cast<const h8*>(srcB[j] + (int64_t)kb * 1024);
      d[j][1] = *reinterpret_cast<const h8*>(srcB[j] + (int64_t)kb * 1024 + 512);
    }
  };
  auto storeA = [&](int st) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<h8*>(&sA[st][(wv + 8 * i) * 512 + 8 * lane]) = ra[i];
  };
  f4 acc[QT][FT];
#pragma unroll
  for (int i = 0; i < QT; ++i)
#pragma unroll
    for (int j = 0; j < FT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // one K step: b = frame fragments of step s, nb = the ring slot that receives step s + 2
  auto step = [&](int s, const h8 (&b)[FT][2], h8 (&nb)[FT][2]) {
    const int st = s & 1;
    // query pieces of step s + 1 into the other stage (read by every wave in step s - 1, which ended at
    // the last barrier), then the loads for step s + 2: query pieces first, so the wait for them at the
    // next step leaves the frame fragments of s + 2 in flight
    // (branch-free: past the end the loads repeat the last step and the store fills a stage nobody reads
    // again — a conditional load would make the compiler's vmcnt merge wait for the new loads too)
    if constexpr (X != 4) {
      storeA(st ^ 1);
      loadA(s + 2 < KB ? s + 2 : KB - 1);
    }
    if constexpr (X != 3) loadB(s + D < KB ? s + D : KB - 1, nb);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PP) {
      // memory phase: every query fragment of the step into registers, then publish; compute phase: 24 FT
      // MFMAs while the SIMD's other wave runs its memory phase
      h8 af[QT][2];
#pragma unroll
      for (int i = 0; i < QT; ++i) {
        if constexpr (X == 5) {  // diagnostics: no fragment reads
          af[i][0] = b[i % FT][0];
          af[i][1] = b[i % FT][1];
        } else {
          af[i][0] = *reinterpret_cast<const h8*>(&sA[st][(2 * i) * 512 + 8 * lane]);
          af[i][1] = *reinterpret_cast<const h8*>(&sA[st][(2 * i + 1) * 512 + 8 * lane]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (X == 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (X == 1) {  // keep the fragments live without the matrix cores
#pragma unroll
        for (int i = 0; i < QT; ++i)
#pragma unroll
          for (int j = 0; j < FT; ++j) acc[i][j][0] += (float)af[i][0][0] + (float)af[i][1][0] + (float)b[j][0][0] + (float)b[j][1][0];
      } else {
#pragma unroll
        for (int i = 0; i < QT; ++i)
#pragma unroll
          for (int j = 0; j < FT; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][0], b[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][0], b[j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][1], b[j][0], acc[i][j], 0, 0, 0);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (X != 2) asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
      for (int i = 0; i < QT; ++i) {
        const h8 ah = *reinterpret_cast<const h8*>(&sA[st][(2 * i) * 512 + 8 * lane]);
        const h8 al = *reinterpret_cast<const h8*>(&sA[st][(2 * i + 1) * 512 + 8 * lane]);
#pragma unroll
        for (int j = 0; j < FT; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, b[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, b[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, b[j][0], acc[i][j], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };

  loadA(0);
  loadB(0, rb0);
  if constexpr (X == 3) loadB(0, rb2);
  storeA(0);
  loadA(KB > 1 ? 1 : 0);
  if (D == 2) loadB(KB > 1 ? 1 : 0, rb1);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // ping-pong: waves w and w + 4 share a SIMD; group 1 (waves 4-7) runs one barrier phase behind group 0,
  // so each SIMD alternates one wave's memory phase with the other's MFMAs.  A stage is read in the memory
  // phases of step s (group 0 at phase 2s, group 1 at 2s + 1) and rewritten in those of step s + 1 (2s + 2,
  // 2s + 3); each memory phase ends with lgkmcnt(0) + barrier, so no write overtakes a read and every write
  // is published before its first reader.  Group 0 takes one extra barrier at the end: equal counts.
  const int grp = __builtin_amdgcn_readfirstlane(wv >> 2);
  if (PP && grp) asm volatile("s_barrier" ::: "memory");
  int s = 0;
  if constexpr (D == 2) {  // frame fragments two steps ahead: a ring of three
    for (; s + 3 <= KB; s += 3) {
      step(s, rb0, rb2);
      step(s + 1, rb1, rb0);
      step(s + 2, rb2, rb1);
    }
    if (s < KB) step(s, rb0, rb2);
    if (s + 1 < KB) step(s + 1, rb1, rb0);
  } else {  // one step ahead: a ring of two
    for (; s + 2 <= KB; s += 2) {
      step(s, rb0, rb1);
      step(s + 1, rb1, rb0);
    }
    if (s < KB) step(s, rb0, rb1);
  }
  if (PP && !grp) asm volatile("s_barrier" ::: "memory");
  // epilogue: lane holds queries 16 i + 4 (lane >> 4) + r, frames 16 j + (lane & 15) of its wave's columns;
  // the inverse norms are loaded once (ia / ib cover the padded rows; a frame column past them is clamped
  // for the load and never stored)
  const int64_t q0 = qt0 * 16, n0 = nt * TN + (int64_t)wv * 16 * FT;
  const int64_t nrows = ftiles * 16;
  double ic[FT];
#pragma unroll
  for (int j = 0; j < FT; ++j) {
    const int64_t n = n0 + 16 * j + (lane & 15);
    ic[j] = a.ib[n < nrows ? n : nrows - 1];
  }
  // EP 1 (even N): each 16-query row block goes through the wave's LDS slice (16 x 16 FT f64, row-major)
  // and leaves as 16-byte stores of two adjacent frames; EP 0 (or odd N, whose rows are not all 16-byte
  // aligned): 8-byte stores straight from the accumulator layout
  const bool wide = EP == 1 && (a.N & 1) == 0;
  double* stage = reinterpret_cast<double*>(smem) + wv * 16 * 16 * FT;
#pragma unroll
  for (int i = 0; i < QT; ++i) {
    const int64_t qb = q0 + 16 * i + 4 * (lane >> 4);
    const double4 iq4 = *reinterpret_cast<const double4*>(a.ia + qb);
    const double iqv[4] = {iq4.x, iq4.y, iq4.z, iq4.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t q = qb + r;
      const double iq = iqv[r];
#pragma unroll
      for (int j = 0; j < FT; ++j) {
        const int64_t n = n0 + 16 * j + (lane & 15);
        const double cs = (double)acc[i][j][r] * iq * ic[j];
        const double v = (iq != 0.0 && ic[j] != 0.0) ? (cs + 1.0) / 2.0 : 0.0;
        if constexpr (EP == 2) {  // diagnostics: no stores (wrong output; A/B of the epilogue's cost)
          if (v == -1.0) a.out[0] = v;
        } else if constexpr (EP == 3) {  // float32 scores: the f64 value rounded once
          if (q < a.Q && n < a.N) __builtin_nontemporal_store((float)v, a.outf + q * a.N + n);
        } else if (wide) {
          stage[(4 * (lane >> 4) + r) * 16 * FT + 16 * j + (lane & 15)] = v;
        } else if (q < a.Q && n < a.N) {
          __builtin_nontemporal_store(v, a.out + q * a.N + n);  // write-once scores
        }
      }
    }
    if (wide) {
      // 16 rows x 8 FT pairs of frames; lane c takes pairs c, c + 64, ...
#pragma unroll
      for (int u = 0; u < (16 * 8 * FT + 63) / 64; ++u) {
        const int c = lane + 64 * u;
        if (c >= 16 * 8 * FT) break;
        const int row = c / (8 * FT), pr = c % (8 * FT);
        const int64_t q = q0 + 16 * i + row, n = n0 + 2 * pr;
        const d2v v2 = *reinterpret_cast<const d2v*>(stage + row * 16 * FT + 2 * pr);
        if (q < a.Q) {
          if (n + 1 < a.N) __builtin_nontemporal_store(v2, reinterpret_cast<d2v*>(a.out + q * a.N + n));
          else if (n < a.N) __builtin_nontemporal_store(v2.x, a.out + q * a.N + n);
        }
      }
    }
  }
}

template <int FT, int PP, int D = 2, int EP = 0, int X = 0>
static int launch_t(CosArgs a, hipStream_t s) {
  constexpr int TN = 8 * 16 * FT;
  const int64_t np_rows = a.ntiles * kCosT;
  a.qtiles = (int)(hq_cos_padded_rows(a.Q) / 128);
  a.ntiles = (np_rows + TN - 1) / TN;
  const int64_t nt8 = ((a.ntiles + 7) / 8) * 8;
  const int64_t blocks = nt8 * a.qtiles;
  if (blocks > 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "too many tiles");
  auto kern = k_cos_t<FT, PP, D, EP, X>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(512), 0, s, a, np_rows / 16);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int TN, int PP, bool NTS = true>
static int launch_g3(CosArgs a, hipStream_t s) {
  const int64_t np_rows = a.ntiles * kCosT;
  a.qtiles = (int)(hq_cos_padded_rows(a.Q) / 128);
  a.ntiles = (np_rows + TN - 1) / TN;
  const int64_t nt8 = ((a.ntiles + 7) / 8) * 8;
  const int64_t blocks = nt8 * a.qtiles;
  if (blocks > 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "too many tiles");
  const size_t lds = sizeof(_Float16) * 3 * (2 * 128 + 2 * TN) * kCosK;
  auto kern = k_cos_g3<TN, PP, NTS>;
  HQ_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(TN * 2), lds, s, a, np_rows);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

template <int TQ>
static int launch_cos(CosArgs a, hipStream_t s) {
  a.qtiles = (int)((hq_cos_padded_rows(a.Q) + TQ - 1) / TQ);
  const int64_t nt8 = ((a.ntiles + 7) / 8) * 8;
  const int64_t blocks = nt8 * a.qtiles;
  if (blocks > 0x7FFFFFFF) return fail(HQ_E_UNSUPPORTED, "too many tiles");
  const size_t lds = sizeof(_Float16) * 2 * (2 * TQ + 2 * kCosT) * kCosRow;
  HQ_CHECK_HIP(hipFuncSetAttribute((const void*)k_cos_mfma<TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_cos_mfma<TQ>, dim3((unsigned)blocks), dim3(256), lds, s, a);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

}  // namespace hq

using namespace hq;

extern "C" {

int hq_cos_padded_k(int K) { return K <= 0 ? 0 : ((K + kCosK - 1) / kCosK) * kCosK; }
int64_t hq_cos_padded_rows(int64_t N) { return N <= 0 ? 0 : ((N + kCosT - 1) / kCosT) * kCosT; }

int hq_cos_prepare(const float* X, int64_t N, int64_t ld, int K, void* X16, double* inv, hq_stream_t stream) {
  if (N < 0 || K <= 0 || ld < K) return fail(HQ_E_INVALID, "bad shape N=%lld K=%d ld=%lld", (long long)N, K, (long long)ld);
  if (N == 0) return HQ_OK;
  if (!X || !X16 || !inv) return fail(HQ_E_INVALID, "null buffer");
  const int Kp = hq_cos_padded_k(K);
  const int64_t rows = hq_cos_padded_rows(N);
  // the row-major layout only for the superseded A/B kernels (option cos_kernel 1-3): one wave per row;
  // the tiled layout: one wave per 16-row tile
  const int64_t ek = opt(OPT_COS_KERNEL, 0);
  const bool rowmajor = ek >= 1 && ek <= 3;
  int64_t blocks = rowmajor ? (rows + 3) / 4 : rows / 16;
  if (blocks > 65536) blocks = 65536;
  // tiled: split the K steps over up to 8 workgroups per tile while there are fewer than 1024 tiles
  int parts = 1;
  while (!rowmajor && parts < 8 && blocks * parts < 1024 && (Kp / kCosK) / (2 * parts) >= 16) parts *= 2;
  if (rowmajor)
    hipLaunchKernelGGL(k_cos_prepare, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, X, N, ld, K, Kp, rows,
                       reinterpret_cast<_Float16*>(X16), inv);
  else
    hipLaunchKernelGGL(k_cos_prepare_tiled, dim3((unsigned)blocks, (unsigned)parts), dim3(1024), 0, (hipStream_t)stream,
                       X, N, ld, K, Kp, rows, reinterpret_cast<_Float16*>(X16), inv);
  HQ_CHECK_LAUNCH();
  return HQ_OK;
}

int hq_cos_scores_mfma_f32(const void* A16, const double* inv_a, int Q, const void* B16, const double* inv_b, int64_t N,
                           int K, float* out, hq_stream_t stream) {
  if (Q < 0 || N < 0 || K <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || N == 0) return HQ_OK;
  if (!A16 || !inv_a || !B16 || !inv_b || !out) return fail(HQ_E_INVALID, "null buffer");
  CosArgs a;
  a.A = reinterpret_cast<const _Float16*>(A16);
  a.B = reinterpret_cast<const _Float16*>(B16);
  a.ia = inv_a;
  a.ib = inv_b;
  a.Q = Q;
  a.N = N;
  a.Kp = hq_cos_padded_k(K);
  a.ntiles = hq_cos_padded_rows(N) / kCosT;
  a.out = nullptr;
  a.outf = out;
  return launch_t<3, 1, 1, 3>(a, (hipStream_t)stream);  // the default kernel, float32 score stores
}

int hq_cos_scores_mfma(const void* A16, const double* inv_a, int Q, const void* B16, const double* inv_b, int64_t N,
                       int K, double* out, hq_stream_t stream) {
  if (Q < 0 || N < 0 || K <= 0) return fail(HQ_E_INVALID, "bad shape");
  if (Q == 0 || N == 0) return HQ_OK;
  if (!A16 || !inv_a || !B16 || !inv_b || !out) return fail(HQ_E_INVALID, "null buffer");
  CosArgs a;
  a.A = reinterpret_cast<const _Float16*>(A16);
  a.B = reinterpret_cast<const _Float16*>(B16);
  a.ia = inv_a;
  a.ib = inv_b;
  a.Q = Q;
  a.N = N;
  a.Kp = hq_cos_padded_k(K);
  a.ntiles = hq_cos_padded_rows(N) / kCosT;
  a.out = out;
  a.outf = nullptr;
  // A/B (option cos_kernel): 1 register-staged two-buffer kernel, 2 lockstep (the DMA kernel without the
  // ping-pong stagger), 3 temporal score stores; DESIGN.md §4.5 has the measurements
  const int64_t ek = opt(OPT_COS_KERNEL, 0);
  if (ek == 1) return launch_cos<128>(a, (hipStream_t)stream);
  if (ek == 2) return launch_g3<256, 0>(a, (hipStream_t)stream);
  if (ek == 3) return launch_g3<256, 1>(a, (hipStream_t)stream);
  // tiled-layout forms: 4 lockstep 128 x 256, 5 ping-pong 128 x 128, 6 ping-pong 128 x 256
  // with frame fragments two steps ahead, 7 the same one step ahead, 8 the default with 16-byte score
  // stores through LDS
  if (ek == 4) return launch_t<2, 0>(a, (hipStream_t)stream);
  if (ek == 5) return launch_t<1, 1>(a, (hipStream_t)stream);
  if (ek == 6) return launch_t<2, 1, 2>(a, (hipStream_t)stream);
  if (ek == 7) return launch_t<2, 1, 1>(a, (hipStream_t)stream);
  if (ek == 8) return launch_t<3, 1, 1, 1>(a, (hipStream_t)stream);
#ifdef HQ_DIAG
  if (ek == 90) return launch_t<3, 1, 1, 2>(a, (hipStream_t)stream);  // no score stores (wrong output)
  // diagnostics (wrong output): 91 no MFMAs, 92 no K-loop barriers, 93 no frame loads, 94 no query
  // staging, 95 no query fragment reads
  if (ek == 91) return launch_t<3, 1, 1, 0, 1>(a, (hipStream_t)stream);
  if (ek == 92) return launch_t<3, 1, 1, 0, 2>(a, (hipStream_t)stream);
  if (ek == 93) return launch_t<3, 1, 1, 0, 3>(a, (hipStream_t)stream);
  if (ek == 94) return launch_t<3, 1, 1, 0, 4>(a, (hipStream_t)stream);
  if (ek == 95) return launch_t<3, 1, 1, 0, 5>(a, (hipStream_t)stream);
#endif
  return launch_t<3, 1, 1>(a, (hipStream_t)stream);
}

}  // extern "C"
