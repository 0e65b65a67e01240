/* hq_mi355x.h — C-ABI of libhq_mi355x.so, the MI355X (gfx950) hot path of hilbert_quantization.
 *
 * The reference (Tylerlhess/hilbert-quantization v1.3.0) is pure Python/NumPy and has no FFI: its
 * plugin boundary is a set of Python ABCs injected into the pipelines.  Each entry
 * point below replaces the arithmetic behind one of those ABC methods; the Python package
 * `hq_mi355x` (hilbert-quantization_amd/hq_mi355x) binds them with ctypes and keeps the reference's
 * method names, argument meaning, exceptions and messages.  Replaced reference interfaces are cited
 * as file:line in the reference's `hilbert_quantization/` tree.
 *
 * Conventions (all entry points):
 *   - every buffer argument is a caller-owned DEVICE pointer; nothing here allocates device memory
 *     (hq_scan_topk takes a caller-sized workspace: hq_scan_workspace_size);
 *   - `stream` is a hipStream_t (NULL = default stream); calls are asynchronous on that stream;
 *   - return HQ_OK (0) or a negative HQ_E_* code; hq_last_error() is thread-local;
 *   - no global mutable state: calls are re-entrant from any host thread.
 */
#ifndef HQ_MI355X_H
#define HQ_MI355X_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* hq_stream_t; /* hipStream_t */

/* error codes */
#define HQ_OK 0
#define HQ_E_INVALID (-1)     /* bad argument (shape, pointer, size) */
#define HQ_E_NOT_POW2 (-2)    /* grid side is not a positive power of two */
#define HQ_E_TOO_MANY (-3)    /* more values than n*n cells */
#define HQ_E_HIP (-4)         /* HIP runtime / launch error */
#define HQ_E_UNSUPPORTED (-5) /* valid request outside what this build implements */

/* dtype codes (element type of copy-only buffers) */
#define HQ_F32 0
#define HQ_F64 1
#define HQ_F16 2
#define HQ_BF16 3
#define HQ_I8 4
#define HQ_U8 5
#define HQ_I16 6
#define HQ_I32 7
#define HQ_I64 8

int hq_version(void);
const char* hq_last_error(void);

/* ---- kernel-variant options (parity tests and A/B only) ------------------------------------------
 * Every entry point runs its tuned kernel by default and a default build never reads the environment.
 * hq_set_option selects an alternative form of a kernel (same results, checked by the parity tests):
 * e.g. "fused_v" (fused-kernel variant bits), "fused_generic", "chunk_generic", "chunk_exactdiv",
 * "chunk_wpb", "chunk_cpw", "precomp_grid", "precomp_tree_lds", "cos_kernel" (1 register-staged,
 * 2 lockstep), "refine_global", "select_2stage", "level_scores_v1" (the one-thread-per-pair dense scorer),
 * "scan_split3" (the level-0 scan's pre-filter on the three-MFMA split contraction instead of hi.hi),
 * "scan_occ" (3 (default) / 4 / 5 / 6: the level-0 scan's register target in waves per SIMD), "scanov_split3" (the
 * overall scan's pre-filter on the split contraction), "ov_occ" (2 / 3 / 4: the overall scan's target),
 * "sample_hi" (1: the sample passes' step loops on hi.hi with a split-G epilogue),
 * "sample_kth" (0 = provable bound), "scan_v1" (the
 * LDS-tiled level-0 scan), "scan_variant", "scan_wpb" (4 = four waves per level-0 scan block), "scan_pf" (prefetch
 * distance 2, 3, 4, 6 or 8; default 6 at scan_occ 3, else 4), "sample_variant" (1 = the full-filter sample pass),
 * "rank_ct" (0: the long-list re-rank's runtime level structure; 2: the compile-time one in the short-list kernel too),
 * "rank_win" (0: the long-list ranking by the bitonic sort alone, no window ranking), "rank_sort_nt" (512: lists
 * > 512 in 512-thread workgroups), "rank_sort_small" (0: lists <= 128 in the 1024-entry workgroup).  Options are
 * process-wide: set them before launching, not
 * while other host threads launch.  hq_reset_option restores the default; hq_get_option returns 1 when
 * the option is set (value in *value), 0 when it is at its default, HQ_E_INVALID for an unknown name.
 * hq_diag_build() = 1 for a `make DIAG=1` library (diagnostics kernels; HQ_<NAME> environment variables
 * are read once at load).                                                                         */
int hq_set_option(const char* name, int64_t value);
int hq_reset_option(const char* name);
int hq_get_option(const char* name, int64_t* value);
int hq_diag_build(void);
/* DIAG builds: bounds violations counted by the guarded corpus-row loads of the level-0 scan (k_scan0f,
 * k_sample_topf, k_pool_select; the load is clamped instead of faulting) since the library loaded, and
 * the source line of the first.  Synchronises the device.  Default builds report 0.                  */
int hq_diag_violations(int64_t* count, int* first_line);
/* Launch geometry of the level-0 scan k_scan0f (host only): query blocks of 64, corpus chunks (a multiple
 * of 8: XCD map) of chunk_len rows (a multiple of 16), and the row counts of the split copies it reads
 * (Z16: z_rows = round_up(N, 16) + 48 rows of 64 halves in the tiled fragment layout, S32: s_rows =
 * round_up(N, 4) + 48).  A C caller of hq_seg_pack0_split allocates z_rows x 64 halves and s_rows x 4
 * floats; hq_scan0_geometry(1, N, ...) returns both.  Exported for the bounds test.                 */
int hq_scan0_geometry(int Q, int64_t N, int* nqb, int* nchunks, int64_t* chunk_len, int64_t* z_rows,
                      int64_t* s_rows);

/* ---- M1/M2/M4: coordinate tables ------------------------------------------------------------
 * replaces core/hilbert_mapper.py:17-40 generate_hilbert_coordinates (+ :42-113 d2xy/xy2d/rotate)
 * and rag/embedding_generation/hilbert_mapper.py:122-204.
 * xs, ys: int32[n*n] in curve order (d2xy); xy2d: int32[n*n] row-major (index of cell (x,y) at
 * y*n+x).  Any of the three may be NULL.                                                        */
int hq_hilbert_table(int n, int32_t* xs, int32_t* ys, int32_t* xy2d, hq_stream_t stream);

/* ---- M5: 1-D -> 2-D scatter ---------------------------------------------------------------
 * replaces core/hilbert_mapper.py:115-174 map_to_2d (and rag/.../hilbert_mapper.py:16-75).
 * in: N rows of d elements (row stride in_stride elements); out: N x n x n row-major (row = y),
 * out[y][x] = in[i] for the i with d2xy(i) = (x,y), i < d; zero elsewhere.  Bit copy, any dtype.  */
int hq_map_to_2d(int dtype, const void* in, int64_t N, int64_t in_stride, int d, int n, void* out,
                 hq_stream_t stream);

/* ---- M6: 2-D -> 1-D gather ----------------------------------------------------------------
 * replaces core/hilbert_mapper.py:176-205 map_from_2d (and rag/.../hilbert_mapper.py:77-120,
 * rag/embedding_generation/reconstructor.py:100-131).  img: N x n x n; out: N x d_out with
 * out[i] = img[y_i][x_i], d_out <= n*n (callers truncate, core/pipeline.py:219).               */
int hq_map_from_2d(int dtype, const void* img, int64_t N, int n, int d_out, void* out,
                   hq_stream_t stream);

/* ---- I1: streaming hierarchical index ------------------------------------------------------
 * replaces core/streaming_index_builder.py:315-343 StreamingHilbertIndexGenerator.
 * generate_optimized_indices(image, L) (default index of HilbertQuantizer, core/pipeline.py:59-63).
 * img: N x n x n (dtype HQ_F32 or HQ_F64); the tree is built over the first stream_len values of
 * the Hilbert-ordered stream (n*n for generate_optimized_indices; len(parameters) for
 * generate_indices_during_mapping, :287-313, where partial groups of 4 never promote).
 * idx_out: float64 N x L.                                                                       */
int hq_index_streaming(int dtype, const void* img, int64_t N, int n, int stream_len, int L,
                       double* idx_out, hq_stream_t stream);

/* ---- I2: traditional index -----------------------------------------------------------------
 * replaces core/index_generator.py:313-356 _generate_traditional_indices (used by the chunk
 * encoder, core/streaming_processor.py:858-860,897-899).  img: f32 N x n x n; out: f32 N x L.   */
int hq_index_traditional_f32(const float* img, int64_t N, int n, int L, float* out,
                             hq_stream_t stream);

/* ---- I2/I4 building block: block means ---------------------------------------------------------
 * np.mean of each (n/grid)^2 block of N x n x n images (dtype HQ_F32 or HQ_F64, NumPy pairwise
 * order in that dtype, result in that dtype):
 * order 0 = row-major sections (core/index_generator.py:100-144 calculate_spatial_averages);
 * order 1 = the RAG generator's Hilbert order (hierarchical_index_generator.py:204-244).
 * out: N x cnt with cnt = grid*grid (1 = whole-image mean when grid > n).                       */
int hq_block_means(int dtype, const void* img, int64_t N, int n, int grid, int order, void* out,
                   hq_stream_t stream);

/* ---- I4: RAG multi-row index ---------------------------------------------------------------
 * replaces rag/embedding_generation/hierarchical_index_generator.py:103-146
 * generate_multi_level_indices.  img: f32 N x n x n; out: f32 N x (n + R) x n where
 * R = hq_rag_index_rows(n) (image copied, one row per granularity appended, zero filled).       */
int hq_rag_index_rows(int n);
int hq_index_rag_f32(const float* img, int64_t N, int n, float* out, hq_stream_t stream);

/* ---- Q1/Q2: uint8 quantize / de-normalise ---------------------------------------------------
 * replaces core/compressor.py:256-280 _normalize_for_compression and :282-303
 * _denormalize_from_compression.  enh: f32 N x rows x cols; out u8 same shape;
 * minmax: f32 N x 2 (min, max) written.  Constant images give 128 everywhere.                  */
int hq_quantize_u8(const float* enh, int64_t N, int rows, int cols, uint8_t* out, float* minmax,
                   hq_stream_t stream);
int hq_dequantize_u8(const uint8_t* u8, int64_t N, int rows, int cols, const float* minmax,
                     float* out, hq_stream_t stream);

/* ---- fused map + streaming index + embed + uint8 quantize (the north-star kernel) -----------
 * replaces the component sequence of core/pipeline.py:97-146 quantize_model up to the codec:
 * pad (:325-349) -> map_to_2d -> streaming index (L) -> embed_indices_in_image
 * (core/index_generator.py:221-253) -> _normalize_for_compression.
 * in: f32 N x d (row stride in_stride elements), d <= n*n, 2 <= n <= 128;
 * frame: u8 N x (n+1) x n; idx: f64 N x L (may be NULL); minmax: f32 N x 2 (may be NULL).      */
int hq_map_index_quantize(const float* in, int64_t N, int64_t in_stride, int d, int n, int L,
                          uint8_t* frame, double* idx, float* minmax, hq_stream_t stream);

/* ---- config 5: f16 parameter stream, chunked (core/streaming_processor.py:539-582,877-972) ---
 * Consecutive chunks of `chunk` fp16 values (the last may be shorter, >= chunk/2) are each padded
 * to n*n (n = side of chunk), Hilbert-mapped, given the TRADITIONAL index (L = min(chunk, n)),
 * embedded and quantized: frame u8 nchunks x (n+1) x n, idx f32 nchunks x L, minmax f32 x 2.     */
int hq_chunk_encode_f16(const uint16_t* in, int64_t total, int chunk, uint8_t* frame, float* idx,
                        float* minmax, hq_stream_t stream);

/* ---- S2: level structure of an index vector of length L (host function) -------------------
 * replaces core/search_engine.py:42-109 _parse_index_structure.  Writes up to max_levels rows of
 * (grid, start, end, is_offset) into out[4*max_levels]; returns the number of levels.           */
int hq_parse_structure(int L, int32_t* out, int max_levels);

/* ---- S3 support: per-segment statistics of index vectors -----------------------------------
 * Level segments are those of hq_parse_structure(L).  Vectors are stored "segment padded": segment s
 * starts at a multiple of 4 and is zero-filled to a multiple of 4, Lp = hq_seg_padded_len(L)
 * columns, nseg = hq_seg_count(L).  For every row of idx (f64 N x L):
 *   Z[row][poff_s + j] = (c_j - mean_s) / std_s   (0 where std_s == 0)     f64 N x Lp
 *   stats[row][s]      = {mean_s, std_s, mean(c^2)_s, aux}                f64 N x nseg x 4
 * mean/std follow NumPy's pairwise summation order so the std == 0 branches of
 * core/search_engine.py:137-147 match bit-for-bit.  aux = 0 for f64 sources.                     */
int hq_seg_count(int L);
int hq_seg_padded_len(int L);
int hq_seg_prepare(const double* idx, int64_t N, int L, double* Z, double* stats, hq_stream_t stream);
/* As hq_seg_prepare; src_f32 != 0 marks rows that hold float32 index vectors (widened to f64).  The
 * reference then runs np.mean / np.std / the normalisation (and, when both sides are float32, the
 * whole score) in float32 (core/search_engine.py:137-189 keep the array dtype).  For such rows
 *   Z = f32((c - mean32) / std32), std = std32 (float32 NumPy order), mean = the f64 mean (the sum of
 *   the float32 z is not 0; with the exact mean, sum q*c = std_q std_c G + m mean_q mean_c holds),
 *   aux = 1 (float32 source; the exact scores recompute the float32 statistics), + 2 when the mean of
 *   squares is outside [2^-100, 2^100] (float32 squares under/overflow: the scans' model does not
 *   hold; callers score such rows on the dense exact path).
 * A segment whose float32 std is 0 stores the float32 mean and std 0 (the reference's constant
 * branch, whose mean comparison is float32).                                                     */
int hq_seg_prepare_src(const double* idx, int64_t N, int L, int src_f32, double* Z, double* stats,
                       hq_stream_t stream);
/* As hq_seg_prepare_src with a per-row flag (pools mixing float32 and float64 index vectors):
 * row_f32 (device u8[N], may be NULL: src_f32 applies to every row) != 0 marks float32 rows.      */
int hq_seg_prepare_rows(const double* idx, int64_t N, int L, int src_f32, const uint8_t* row_f32, double* Z,
                        double* stats, hq_stream_t stream);

/* ---- S3/S4: dense EXACT scores ---------------------------------------------------------------
 * replaces core/search_engine.py:111-189 compare_indices_at_level (level >= 0) and :191-230
 * _calculate_overall_similarity (level == -1) for Q queries against N candidates of equal L.
 * Scores are evaluated in the reference's operation order (products and squared differences
 * summed in NumPy's pairwise order), so they are bit-identical to the reference.  Inputs per side:
 * the raw index vectors R (f64 x L) and their hq_seg_prepare outputs (Z, S).  scores: f64 Q x N. */
int hq_level_scores(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                    const double* Zc, const double* Sc, int64_t N, int L, int level, double* scores,
                    hq_stream_t stream);

/* ---- S5/S6: fused MFMA scan with per-query top-k (APPROXIMATE scores) ------------------------
 * One pass over the corpus: f64 MFMA contraction (v_mfma_f64_16x16x4f64) of the normalised
 * vectors + algebraic score epilogue (|score - exact| < 1e-12 for L <= 64) + per-query top-k by
 * (score desc, id asc).  mode 0: level-0 score (progressive filter, search_engine.py:232-300;
 * video hierarchical scan, core/video_search.py:215-264); mode 1: overall score
 * (brute_force_search :302-338).  thr_mode 0: keep all; 1: score >= threshold; 2: > threshold.
 * Also the first arg-max of the approximate score (out_best, may be NULL).  id_base is added to
 * local row ids (sharding).  out_score/out_id: Q x k (-inf / -1 in empty slots), 1 <= k <= 64.
 * The exact ranking is obtained with hq_refine_topk on a slightly larger list.  Vectors with an aux
 * bit 2 (unsafe) segment are outside the model: callers use the dense exact path for them.  Mode 0
 * without the arg-max and with a level-0 segment of <= 32 values runs an f64 wave-level kernel for
 * f64 sources only (float32 rows: hq_scan0_topk_split).
 * workspace: hq_scan_workspace_size(Q, N, k) bytes of device memory.                            */
size_t hq_scan_workspace_size(int Q, int64_t N, int k);
int hq_scan_topk(const double* Zq, const double* Sq, int Q, const double* Zc, const double* Sc,
                 int64_t N, int L, int mode, int k, double threshold, int thr_mode, int64_t id_base,
                 void* workspace, size_t workspace_bytes, double* out_score, int64_t* out_id,
                 double* out_best, int64_t* out_best_id, hq_stream_t stream);

/* ---- S5/S6 level-0 scan on the matrix cores (the progressive search's filtering stage) ----------
 * Same result contract as hq_scan_topk(mode 0, no arg-max), but the contraction G = sum zq*zc runs as
 * a split-f16 product (z = hi + lo, G ~= hi.hi + hi.lo + lo.hi with f32 accumulation, three
 * v_mfma_f32_16x16x32_f16 per 16x16 tile) and the filter and list scores in f32.
 * |approx - exact| <= ~5.5e-6, so callers re-rank with hq_refine_topk at eps >= 2e-5.
 * hq_seg_pack0_split builds, from hq_seg_prepare's Z and S, Z16: f16 hi[32], lo[32] of the
 * zero-padded level-0 segment for round_up(N, 16) + 48 rows (128 B per row), in 16-row tiles of 2 KiB:
 * [hi: 64 x 8][lo: 64 x 8] halves, the 8 at (16 g + j) * 8 being row 16 t + j, values 8 g .. 8 g + 7
 * (one MFMA operand fragment per lane: a wave loads 1 KiB of consecutive bytes), and S32, f32 statistics (std, mean, msq, flag bits) in SoA
 * groups of 4 rows (std[4], mean[4], msq[4], flags[4]) for round_up(N, 4) + 48 rows (16 B per row);
 * Sq/Sc are the f64 statistics of hq_seg_prepare.  Level-0 segments of up to 32 values, N < 2^31. */
/* Starting threshold of hq_scan0_topk_split: the K'-th best score of a 1/16 sample (every 16th tile of
 * 16 rows) minus the error
 * margin, K' = the smallest count with P(Binomial(k, 1/16) >= K') <= 1e-7 (12 at k = 28, 24 at k = 108,
 * 107 at k = 1008; option sample_kth overrides; K' = k, a provable lower bound of the k-th best, for
 * corpora below 16 x 4096 rows).  k up to 1024: lists longer than 64 (the reference engine's default
 * max_candidates_per_level = 100, SearchConfig's 1000) are reduced by a per-query LDS sort of the pool,
 * whose capacity is sized from the sample (an overflowing pool marks its query unresolved).  With K' < k a query can end with fewer than k listed candidates although more pass
 * the caller's threshold: its empty slots then carry score +inf (id -1), which hq_refine_topk /
 * hq_refine_rescore_topk report as unresolved (the caller's dense exact path answers the query).    */
/* hq_seg_prepare_pack0: hq_seg_prepare_rows + hq_seg_pack0_split in one launch (query batches: one wave
 * per row, the same arithmetic and outputs as the two calls; L <= 4096, level-0 segment <= 32 values).  */
int hq_seg_prepare_pack0(const double* idx, int64_t N, int L, int src_f32, const uint8_t* row_f32, double* Z,
                         double* stats, void* Z16, float* S32, hq_stream_t stream);
int hq_seg_level0_len(int L);
int hq_seg_pack0_split(const double* Z, const double* S, int64_t N, int L, void* Z16, float* S32,
                       hq_stream_t stream);
int hq_scan0_topk_split(const void* Zq16, const float* Sq32, const double* Sq, int Q, const void* Zc16,
                        const float* Sc32, const double* Sc, int64_t N, int L, int k, double threshold,
                        int thr_mode, int64_t id_base, void* workspace, size_t workspace_bytes,
                        double* out_score, int64_t* out_id, hq_stream_t stream);
/* hq_seg_flag_rows: the rows of a split copy (S32 of hq_seg_pack0_split) whose zero-variance / f32-unsafe
 *   flag is set, listed once per corpus into flags [1 + N] int32: flags[0] = count, then the rows (any
 *   order).  hq_scan0_topk_split_fl: hq_scan0_topk_split with that list of the corpus (the plain entry
 *   lists the flagged rows on every call: one memset and one pass over S32 per query batch).           */
int hq_seg_flag_rows(const float* S32, int64_t N, int* flags, hq_stream_t stream);
int hq_scan0_topk_split_fl(const void* Zq16, const float* Sq32, const double* Sq, int Q, const void* Zc16,
                           const float* Sc32, const double* Sc, int64_t N, int L, int k, double threshold,
                           int thr_mode, int64_t id_base, void* workspace, size_t workspace_bytes,
                           double* out_score, int64_t* out_id, const int* corpus_flags, hq_stream_t stream);

/* ---- S5 brute force: split-f16 overall scan ----------------------------------------------------
 * Replaces the per-candidate _calculate_overall_similarity loop of brute_force_search
 * (core/search_engine.py:302-338, :191-230) with one scan over all levels: approximate overall scores
 * (|approx - exact| <= ~6e-6) -> per-query top k, re-ranked exactly by hq_refine_topk (mode 1).
 * hq_seg_packov_info: the layout of L's level segments (K-blocks of 32 values, segments of >= 2 values,
 * one-value segments, floats per statistics group of 4 rows); HQ_E_UNSUPPORTED when L has none (a
 * segment longer than 32 values, more than 4 / 2 of either kind, or another block pattern than the
 * L = 64 and L = 32 structures): callers keep hq_scan_topk.
 * hq_seg_packov_split builds from hq_seg_prepare's Z and S: Zo16, f16 hi / lo of every segment's
 * normalised values packed into the K-blocks, round_up(N, 16) + 48 rows of nkb x 128 B in 16-row
 * tiles of nkb x 2 KiB (hq_seg_pack0_split's fragment order per block), and So32, f32 statistics in
 * groups of 4 rows (per one-value segment value[4], row flags[4], pre-filter offsets[4], then per row
 * and segment (std, mean, msq, zero-std flag)) for (round_up(N, 4) + 48) / 4 groups.
 * hq_scanov_topk_split: Zq/Zc are hq_seg_prepare's f64 Z (rows with an f32-unsafe statistic are scored
 * from them in f64); the starting threshold comes from a 1/16 tile sample (K' as
 * hq_scan0_topk_split: short lists carry +inf, which hq_refine_topk reports as unresolved).  k <= 1024. */
int hq_seg_packov_info(int L, int* nkb, int* ng, int* nc, int* group_floats);
int hq_seg_packov_split(const double* Z, const double* S, int64_t N, int L, void* Zo16, float* So32,
                        hq_stream_t stream);
size_t hq_scanov_workspace_size(int Q, int64_t N, int k);
int hq_scanov_topk_split(const void* Zq16, const float* Sq32, const double* Sq, const double* Zq, int Q,
                         const void* Zc16, const float* Sc32, const double* Sc, const double* Zc, int64_t N, int L,
                         int k, double threshold, int thr_mode, int64_t id_base, void* workspace,
                         size_t workspace_bytes, double* out_score, int64_t* out_id, hq_stream_t stream);

/* ---- S5/S6: exact re-rank of a scan list -----------------------------------------------------
 * cand_score/cand_id: Q x kp list from hq_scan_topk (approximate, sorted).  Re-scores every listed
 * candidate exactly (as hq_level_scores), applies the threshold test exactly and writes the exact
 * top-k (score desc, id asc): out_score/out_id Q x k, out_count Q, and out_resolved Q = 1 when the
 * result is provably the exact top-k over the whole corpus given |approx - exact| <= eps (else the
 * caller re-runs that query on the dense exact path).  kp <= 1024 (lists longer than 64 are staged in
 * tiles and ranked by an LDS sort; even L), k <= kp.  out_redo (device int, may
 * be NULL): the number of queries that need the dense path — unresolved, or (count_empty != 0) with
 * no candidate passing — so the caller syncs on one int.                                          */
int hq_refine_topk(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                   const double* Zc, const double* Sc, int64_t N, int L, int mode,
                   const double* cand_score, const int64_t* cand_id, int kp, int k,
                   double threshold, int thr_mode, double eps, int64_t id_base, double* out_score,
                   int64_t* out_id, int* out_count, int* out_resolved, int count_empty, int* out_redo,
                   hq_stream_t stream);
/* hq_refine_topk + the exact re-score of its output (core/search_engine.py:191-230 for each output
 * pair, as hq_rescore computes it): out_det [Q, k, 1 + nseg] = [overall, level 0, level 1, ...] of
 * every output entry, zeros for empty slots.  The candidates' rows are staged once per query in LDS,
 * so the progressive search needs no separate hq_rescore launch for its survivors.                  */
int hq_refine_rescore_topk(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                           const double* Zc, const double* Sc, int64_t N, int L, int mode,
                           const double* cand_score, const int64_t* cand_id, int kp, int k,
                           double threshold, int thr_mode, double eps, int64_t id_base,
                           double* out_score, int64_t* out_id, int* out_count, int* out_resolved,
                           int count_empty, int* out_redo, double* out_det, hq_stream_t stream);
/* hq_refine_rescore_topk with a ping-pong pair of redo counters (no memset launch per batch): out_redo
 * must be zero on entry (fresh, or cleared by the previous call as its next_redo); the kernel clears
 * next_redo for the next batch.  Alternate the two counters between consecutive batches of a stream and
 * copy out_redo to the host behind the batch (the next batch's kernels run after that copy).          */
int hq_refine_rescore_topk_pp(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                              const double* Zc, const double* Sc, int64_t N, int L, int mode,
                              const double* cand_score, const int64_t* cand_id, int kp, int k,
                              double threshold, int thr_mode, double eps, int64_t id_base,
                              double* out_score, int64_t* out_id, int* out_count, int* out_resolved,
                              int count_empty, int* out_redo, int* next_redo, double* out_det,
                              hq_stream_t stream);
/* The three entries above in one, with a device workspace (hq_refine_workspace_size bytes; may be NULL):
 * out_det and next_redo nullable (NULL out_det = hq_refine_topk's outputs; a non-NULL next_redo = the
 * ping-pong counters of hq_refine_rescore_topk_pp).  Lists longer than 64 then run the lane-cooperative
 * re-rank: 8 lanes score one list entry (NumPy's eight pairwise accumulators one per lane, the row staged
 * with 16-byte loads), every level of the entry in one pass over its row, the exact scores, ids and records
 * to the workspace, then one workgroup per query ranks them.  Same outputs, bit for bit.
 * Replaces the re-rank arithmetic of core/search_engine.py:232-300 (level-0 filter) and :340-388
 * (overall re-score of the survivors) for the reference's default lists (M = 100, :31; 1000, config.py:181). */
size_t hq_refine_workspace_size(int Q, int kp, int L);
int hq_refine_topk_ws(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                      const double* Zc, const double* Sc, int64_t N, int L, int mode,
                      const double* cand_score, const int64_t* cand_id, int kp, int k,
                      double threshold, int thr_mode, double eps, int64_t id_base,
                      double* out_score, int64_t* out_id, int* out_count, int* out_resolved,
                      int count_empty, int* out_redo, int* next_redo, double* out_det,
                      void* workspace, size_t workspace_bytes, hq_stream_t stream);
/* The level-0 re-rank of one progressive search (mode 0, records on, count_empty on) with its final
 * ranking fused in: the level-0 outputs and the proof as hq_refine_topk_ws (out_det not produced), and
 * fin_id [Q, K_out], fin_det [Q, K_out, 1 + nseg], fin_count [Q] = hq_progressive_final_ex's outputs for
 * R = 1 and no arg-max fallback (best id -1: a query where nothing passed gets count 0 and is counted in
 * out_redo).  The final order is core/search_engine.py:387's stable sort by the overall score over the
 * level-0 order (key32: thr_mode | HQ_THR_KEY32 ranks by float32-rounded keys).  On the lane-cooperative
 * paths only (the cooperative shapes; kp > 64 needs the workspace); HQ_E_UNSUPPORTED otherwise, and the
 * caller keeps the two-step form.  out_score and out_id may both be NULL: the level-0 lists are then not
 * written (the final outputs, count, resolved flag and redo count are the same). */
int hq_refine_final_ws(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
                       const double* Zc, const double* Sc, int64_t N, int L, const double* cand_score,
                       const int64_t* cand_id, int kp, int k, double threshold, int thr_mode, double eps,
                       int64_t id_base, double* out_score, int64_t* out_id, int* out_count,
                       int* out_resolved, int* out_redo, int* next_redo, int K_out, int64_t* fin_id,
                       double* fin_det, int* fin_count, void* workspace, size_t workspace_bytes,
                       hq_stream_t stream);

/* ---- S4 on candidate lists: EXACT overall + per-level scores of selected pairs ---------------
 * ids: int64 Q x k GLOBAL ids (row = id - id_base; out of range / < 0 -> zeros);
 * out: f64 Q x k x (1 + nseg) = [overall, level_0 .. level_{nseg-1}] (search_engine.py:191-230). */
int hq_rescore(const double* Rq, const double* Zq, const double* Sq, int Q, const double* Rc,
               const double* Zc, const double* Sc, int64_t N, int L, const int64_t* ids, int k,
               int64_t id_base, double* out, hq_stream_t stream);

/* ---- S5 final stage, R-way (R = number of corpus shards) -------------------------------------
 * Inputs per shard r: level-0 top-M lists s0/ids (R x Q x M, sorted), their rescored rows det
 * (R x Q x M x (1+nseg)), and the shard's level-0 arg-max best/best_id (R x Q) with its row
 * best_det (R x Q x (1+nseg)).  Forms the global level-0 top-M, falls back to the global first
 * arg-max when no candidate passed (search_engine.py:295-298), stable-sorts the survivors by the
 * overall score (:386-388) and writes the top K: out_id (Q x K, -1 padded), out_det
 * (Q x K x (1+nseg)), out_count (Q).  M <= 1024, R <= 16.                                        */
int hq_progressive_final(int R, int Q, int M, int nseg, const double* s0, const int64_t* ids,
                         const double* det, const double* best, const int64_t* best_id,
                         const double* best_det, int K, int64_t* out_id, double* out_det,
                         int* out_count, hq_stream_t stream);
/* hq_progressive_final with flags: 1 = float32 sort keys (every vector float32: the reference's sort
 * compares a numpy float32 score with a Python-float one in float32 under NumPy 2 / NEP 50, so the merge
 * and the stable sort rank by the float32-rounded values; core/search_engine.py:291, :387).  The re-rank
 * takes the same mode as thr_mode | 8 (HQ_THR_KEY32) on hq_refine_topk / hq_refine_rescore_topk.      */
#define HQ_THR_KEY32 8
int hq_progressive_final_ex(int R, int Q, int M, int nseg, const double* s0, const int64_t* ids,
                            const double* det, const double* best, const int64_t* best_id,
                            const double* best_det, int K, int64_t* out_id, double* out_det,
                            int* out_count, int flags, hq_stream_t stream);

/* ---- S5 support: top-k of a dense score matrix (k > 64, e.g. max_candidates_per_level = 100) -----
 * scores f64 Q x N -> out_score/out_id Q x k ordered (score desc, id asc) among candidates passing
 * thr_mode (0 none, 1 >=, 2 >); out_best/out_best_id (may be NULL): first arg-max.               */
int hq_select_topk(const double* scores, int Q, int64_t N, int k, double threshold, int thr_mode,
                   int64_t id_base, double* out_score, int64_t* out_id, double* out_best,
                   int64_t* out_best_id, hq_stream_t stream);
/* Two-stage form of hq_select_topk for long rows (the dense exact fallback: few queries x a 1M-row
 * corpus): parts of ~8192 entries select their own top-k and arg-max in parallel (one wave each), then
 * one wave per query merges the parts' candidates in the same total order - identical results.
 * workspace: hq_select_workspace_size(Q, N, k) bytes (0 / NULL -> the one-stage kernel).           */
size_t hq_select_workspace_size(int Q, int64_t N, int k);
int hq_select_topk_ws(const double* scores, int Q, int64_t N, int k, double threshold, int thr_mode,
                      int64_t id_base, void* workspace, size_t workspace_bytes, double* out_score,
                      int64_t* out_id, double* out_best, int64_t* out_best_id, hq_stream_t stream);

/* ---- S3 on raw segments (candidate pools of mixed index length) -------------------------------
 * compare_indices_at_level for the level segments already sliced and truncated to a common length
 * m (search_engine.py:122-135): q f64[m] against C f64 N x m -> out f64[N].                      */
int hq_pair_scores_raw(const double* q, const double* C, int64_t N, int m, double* out,
                       hq_stream_t stream);
/* As hq_pair_scores_raw; q_f32 / c_f32 != 0: that side holds float32 values, whose statistics and
 * normalised values the reference computes in float32 (the whole score when both are float32).   */
int hq_pair_scores_raw_src(const double* q, const double* C, int64_t N, int m, int q_f32, int c_f32,
                           double* out, hq_stream_t stream);

/* ---- S7: RAG cosine scores (rag/search/engine.py:622-660, 1025-1051) --------------------------
 * a: f32 Q x K, b: f32 N x K -> out f64 Q x N of (cos + 1) / 2 (0 if a norm is 0).               */
int hq_cosine_scores(const float* a, int Q, const float* b, int64_t N, int K, double* out,
                     hq_stream_t stream);

/* ---- §8f row 3: pre-computed overlapping-square index ---------------------------------------
 * replaces core/precomputed_hilbert_index.py:65-212 PrecomputedHilbertIndexer.
 * create_precomputed_index (built for every model by HilbertQuantizer.quantize, api.py:162-173).
 * hq_precomputed_layout: levels of _calculate_granularity_levels (:121-149) as int32 quadruples
 *   (grid, square, count, first output) into levels_out[4*max_out]; returns the level count.
 * hq_precomputed_index: N inputs -> float32 averages [N, T] (row stride out_stride >= T), levels
 *   finest first, each level = grid squares row-major then the half-offset squares; every value is
 *   float32(np.mean(square)) bit for bit.  kind 0: n x n images (dtype HQ_F32 / HQ_F64, image
 *   stride in_stride elements); kind 1: 1-D Hilbert-ordered streams of d <= n*n values, zero
 *   padded (core/pipeline.py:298-319 _get_2d_representation).  n: power of two <= 128 (f64: <= 64);
 *   max_levels / min_square_size as PrecomputedHilbertIndexer's constructor (defaults 6, 2).        */
int hq_precomputed_layout(int n, int max_levels, int min_square_size, int32_t* levels_out, int max_out);
int hq_precomputed_index(int dtype, int kind, const void* in, int64_t N, int64_t in_stride, int d, int n,
                         int max_levels, int min_square_size, float* out, int64_t out_stride, hq_stream_t stream);
/* hq_precomputed_stats: per vector and level l (averages [offsets[l], offsets[l] + counts[l]) of
 *   each row of avgs, row stride `stride`): stats [N, nlev, 3] float32 = (np.mean, np.std,
 *   np.mean(a**2)) in NumPy's order, and norm (same layout as avgs) = (a - mean) / std where std != 0.
 *   Call it with counts = min(query count, candidate count) per level (the reference truncates,
 *   :427-431).
 * hq_precomputed_similarity: replaces :358-466 (_calculate_precomputed_similarity over
 *   _compare_precomputed_levels) for Q x N pairs: out_overall [Q, N] (float64 holding the exact
 *   value), out_type [Q, N] (0: the reference returns a numpy float32, 1: a Python float — decides
 *   the `>= similarity_threshold` comparison, :342), out_levels [Q, N, nlev] (nullable).  weights:
 *   the normalised level weights (Python floats, :390-404).                                      */
/* hq_pearson_f64: replaces :468-496 (PrecomputedSimilaritySearchEngine.compare_indices_at_level, the
 *   legacy np.corrcoef comparison) for one query q[m] against N rows of C [N, m] -> out [N] f64;
 *   np.std branches and np.allclose exact, the correlation within ~1e-15 (BLAS order in np.cov). */
int hq_pearson_f64(const double* q, const double* C, int64_t N, int m, double* out, hq_stream_t stream);
int hq_precomputed_stats(const float* avgs, int64_t N, int64_t stride, int nlev, const int32_t* offsets,
                         const int32_t* counts, float* stats, float* norm, hq_stream_t stream);
int hq_precomputed_similarity(const float* q_avgs, const float* q_norm, const float* q_stats, int Q, int64_t q_stride,
                              const float* c_avgs, const float* c_norm, const float* c_stats, int64_t N,
                              int64_t c_stride, int nlev, const int32_t* q_offsets, const int32_t* c_offsets,
                              const int32_t* counts, const double* weights, double* out_overall, uint8_t* out_type,
                              double* out_levels, hq_stream_t stream);

/* ---- S7 dense frame similarity on the matrix cores ------------------------------------------
 * replaces rag/search/engine.py:622-660 (_calculate_embedding_cosine_similarity) for Q query x N
 * frame pairs of K values (e.g. 64 x 64 images, K = 4096).
 * hq_cos_prepare: f32 rows X [N, K] (row stride ld) -> split-f16 copies X16 of hq_cos_padded_rows(N) x 2 x
 *   hq_cos_padded_k(K) halves (power-of-two scaled hi / lo halves in 1 KiB MFMA operand fragments: 16-row
 *   tile t, K step kb of 32, plane p at ((t KB + kb) 2 + p) x 512 halves, lane 16 g + j = row 16 t + j,
 *   k = 32 kb + 8 g .. + 7; the superseded kernels of option cos_kernel 1-3 use rows [N, 2, Kp]) and
 *   inv [padded rows] = 1 / (scale |x|) (0 for a zero row).  Prepare a corpus once, each query batch per
 *   call, under the same cos_kernel option as the scoring call.
 * hq_cos_scores_mfma: out [Q, N] f64 = (cos + 1) / 2 (0 when a norm is 0), split-f16 MFMA contraction
 *   (v_mfma_f32_16x16x32_f16 x 3), within 1e-5 of the reference's float32 BLAS result.
 * hq_cos_scores_mfma_f32: the same scores rounded once to float32 (the reference's own score dtype; half
 *   the output bytes).                                                                           */
int hq_cos_padded_k(int K);
int64_t hq_cos_padded_rows(int64_t N);
int hq_cos_prepare(const float* X, int64_t N, int64_t ld, int K, void* X16, double* inv, hq_stream_t stream);
int hq_cos_scores_mfma(const void* A16, const double* inv_a, int Q, const void* B16, const double* inv_b, int64_t N,
                       int K, double* out, hq_stream_t stream);
int hq_cos_scores_mfma_f32(const void* A16, const double* inv_a, int Q, const void* B16, const double* inv_b, int64_t N,
                           int K, float* out, hq_stream_t stream);

/* ---- S7: the rest of the RAG scorer (rag/search/engine.py) --------------------------------------
 * hq_cosine_scores_dt: as hq_cosine_scores for float32 (HQ_F32) or float64 (HQ_F64) rows; float64
 *   inputs are not narrowed (engine.py:622-660 computes in the input dtype).
 * hq_detect_heights: _detect_original_embedding_height (engine.py:134-162) of N images [N, H, W]: the
 *   first row from the bottom with fewer than half zeros ends the original embedding (height = row + 1,
 *   H when none) -> out int32 [N].  _extract_original_embedding (:604-620) is the image's first rows.
 * hq_spatial_locality: _calculate_spatial_locality_similarity (engine.py:662-714) of every query image
 *   q [Q, H, W] against every stored image c [N, H, W] -> out f64 [Q, N]: original heights detected on
 *   both (different -> 0.0), ws = min(4, h / 4, W / 4), one cosine over the block when ws < 2, else the
 *   mean (NumPy pairwise order) of the (cos + 1) / 2 of ws x ws windows at stride ws / 2.  H * W <= 8192.
 * hq_threshold_select: _apply_progressive_threshold (engine.py:243-287) for Q rows of candidate scores
 *   [Q, N] in the caller's order: the first `cap` candidates with score >= threshold -> out_ids [Q, cap]
 *   (ids[q, i] when ids is given, else the position i; -1 padded), out_count [Q].  The caller computes
 *   the level's threshold and cap exactly as the reference (Python float arithmetic).               */
int hq_cosine_scores_dt(int dtype, const void* a, int Q, const void* b, int64_t N, int K, double* out,
                        hq_stream_t stream);
int hq_detect_heights(int dtype, const void* imgs, int64_t N, int H, int W, int* out, hq_stream_t stream);
int hq_spatial_locality(int dtype, const void* q, int Q, const void* c, int64_t N, int H, int W, double* out,
                        hq_stream_t stream);
int hq_threshold_select(const double* scores, const int64_t* ids, int Q, int64_t N, double threshold, int64_t cap,
                        int64_t* out_ids, int64_t* out_count, hq_stream_t stream);

/* ---- §8e: the sharded search's one collective (RCCL over xGMI) ----------------------------------
 * The corpus is split into contiguous global-id ranges, one per GPU (one process per GPU); each rank
 * answers the whole query batch against its shard and packs fixed-size top-k records, and ONE
 * all-gather lets every rank merge them with hq_progressive_final (the reference's analogue: the
 * thread fan-out + list-concatenation merge of core/video_search.py:722-875).
 * hq_comm_unique_id: rank 0 creates the communicator id (HQ_COMM_ID_BYTES opaque bytes) and hands it
 *   to every rank out of band (hq_mi355x.distributed uses the torch.distributed store / broadcast);
 * hq_comm_init_rank: collective over the nranks processes, on the calling thread's current HIP device;
 * hq_allgather_topk: recv [nranks x bytes] = every rank's send [bytes], in rank order, on `stream`;
 *   bytes must be equal on all ranks.  Asynchronous like every other entry point.                   */
#define HQ_COMM_ID_BYTES 128
int hq_comm_unique_id(void* id_out);
int hq_comm_init_rank(void** comm, int nranks, const void* id, int rank);
int hq_comm_size(void* comm, int* nranks, int* rank);
int hq_comm_destroy(void* comm);
int hq_allgather_topk(void* comm, const void* send, void* recv, size_t bytes, hq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HQ_MI355X_H */
