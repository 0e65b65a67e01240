#!/usr/bin/env python3
"""Generate golden vectors by running the REAL reference (hilbert_quantization v1.3.0) on seeded
inputs.  Build-container only: it needs /root/reference, which never travels to the GPU box; the
resulting *.npz files are committed and are pure data (no pickles: np.load(allow_pickle=False)).

    python tests/golden/make_golden.py [--ref /root/reference]

The reference imports cv2 at package import time (core/video_storage.py:19) although none of the
hot-path modules use it, so a do-nothing `cv2` module is placed on sys.path from a temp dir.
"""
import argparse
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference(ref_root):
    stub_dir = tempfile.mkdtemp(prefix="hq_cv2stub_")
    with open(os.path.join(stub_dir, "cv2.py"), "w") as f:
        f.write("# inert stub: the hot-path modules never call cv2\n")
    sys.path[:0] = [stub_dir, ref_root]
    sys.dont_write_bytecode = True
    import logging
    logging.disable(logging.CRITICAL)
    import hilbert_quantization  # noqa: F401
    return hilbert_quantization


def mapper_fixtures(hq):
    from hilbert_quantization.core.hilbert_mapper import HilbertCurveMapper
    from hilbert_quantization.rag.embedding_generation.hilbert_mapper import HilbertCurveMapperImpl
    m = HilbertCurveMapper()
    rm = HilbertCurveMapperImpl(None)
    out = {}
    for n in [1, 2, 4, 8, 16, 32, 64, 128]:
        out[f"coords_n{n}"] = np.array(m.generate_hilbert_coordinates(n), dtype=np.int16).reshape(-1, 2)
    for n in [1, 2, 4, 8, 16, 32, 64]:
        t = np.zeros((n, n), dtype=np.int32)
        for y in range(n):
            for x in range(n):
                t[y, x] = m._xy_to_hilbert_index(x, y, n)
        out[f"xy2d_n{n}"] = t
    rng = np.random.default_rng(1234)
    cases = [(5, 4, np.float32), (16, 4, np.float64), (100, 16, np.float32), (1024, 32, np.float32),
             (1536, 64, np.float32), (700, 32, np.int32), (256, 16, np.float16), (4096, 64, np.float64)]
    for k, (d, n, dt) in enumerate(cases):
        if np.issubdtype(dt, np.integer):
            p = rng.integers(-1000, 1000, size=d).astype(dt)
        else:
            p = rng.standard_normal(d).astype(dt)
        img = m.map_to_2d(p, (n, n))
        out[f"map_in_{k}"] = p
        out[f"map_out_{k}"] = img
        out[f"unmap_out_{k}"] = m.map_from_2d(img)
        out[f"rag_map_out_{k}"] = rm.map_to_2d(p, (n, n))
        out[f"rag_unmap_out_{k}"] = rm.map_from_2d(img)
    return out


def index_fixtures(hq):
    from hilbert_quantization.core.hilbert_mapper import HilbertCurveMapper
    from hilbert_quantization.core.streaming_index_builder import StreamingHilbertIndexGenerator
    from hilbert_quantization.core.index_generator import HierarchicalIndexGeneratorImpl
    from hilbert_quantization.rag.embedding_generation.hierarchical_index_generator import (
        HierarchicalIndexGenerator as RagGen)
    m = HilbertCurveMapper()
    sg = StreamingHilbertIndexGenerator()
    tg = HierarchicalIndexGeneratorImpl()
    rg = RagGen()
    rng = np.random.default_rng(99)
    out = {}
    k = 0
    for (n, L, d) in [(2, 2, 4), (4, 4, 16), (8, 8, 64), (16, 16, 200), (32, 32, 1024), (64, 64, 1536),
                      (32, 20, 1000), (64, 100, 4096), (16, 7, 256), (128, 128, 10000)]:
        p = rng.standard_normal(d).astype(np.float32)
        img = m.map_to_2d(p, (n, n))
        out[f"stream_img_{k}"] = img
        out[f"stream_L_{k}"] = np.int64(L)
        out[f"stream_idx_{k}"] = sg.generate_optimized_indices(img, L)
        k += 1
    k = 0
    for (n, L, d) in [(8, 8, 64), (16, 16, 256), (32, 32, 1024), (64, 64, 1536), (32, 32, 512), (16, 40, 200),
                      (64, 32, 3000)]:
        p = (rng.standard_normal(d) * 3 + 0.5).astype(np.float32)
        img = m.map_to_2d(p, (n, n))
        out[f"trad_img_{k}"] = img
        out[f"trad_L_{k}"] = np.int64(L)
        out[f"trad_idx_{k}"] = tg.generate_optimized_indices(img, L)
        k += 1
    out["trad_alloc_32"] = np.array(tg.calculate_level_allocation(32), dtype=np.int64)
    out["trad_alloc_64"] = np.array(tg.calculate_level_allocation(64), dtype=np.int64)
    k = 0
    for (n, d, dt) in [(16, 256, np.float32), (32, 1024, np.float32), (64, 4096, np.float32),
                       (32, 768, np.float64), (8, 64, np.float32)]:
        p = rng.standard_normal(d).astype(dt)
        img = m.map_to_2d(p, (n, n))
        out[f"rag_img_{k}"] = img
        out[f"rag_rows_{k}"] = rg.generate_multi_level_indices(img)
        k += 1
    return out


def quant_fixtures(hq):
    """cfg2 slice: pad -> map -> streaming index (L = n) -> embed -> uint8 normalise, exactly the
    component sequence of QuantizationPipeline.quantize_model (core/pipeline.py:97-146)."""
    from hilbert_quantization.core.pipeline import QuantizationPipeline
    from hilbert_quantization.core.compressor import MPEGAICompressorImpl
    from hilbert_quantization.core.dimension_calculator import PowerOf4DimensionCalculator
    pipe = QuantizationPipeline(dimension_calculator=PowerOf4DimensionCalculator(min_efficiency_ratio=0.2))
    out = {}
    rng = np.random.default_rng(7)
    for tag, d, N in [("d1536", 1536, 6), ("d1024", 1024, 6), ("d300", 300, 4), ("d4096", 4096, 2)]:
        P = rng.standard_normal((N, d)).astype(np.float32)
        frames, idxs, mins, maxs, enhs = [], [], [], [], []
        for i in range(N):
            p = P[i]
            dims = pipe.dimension_calculator.calculate_optimal_dimensions(len(p))
            pc = pipe.dimension_calculator.calculate_padding_strategy(len(p), dims)
            pp = pipe._pad_parameters(p, dims, pc)
            img = pipe.hilbert_mapper.map_to_2d(pp, dims)
            idx = pipe.index_generator.generate_optimized_indices(img, dims[0])
            enh = pipe.index_generator.embed_indices_in_image(img, idx)
            comp = MPEGAICompressorImpl()
            u8 = comp._normalize_for_compression(enh)
            frames.append(u8)
            idxs.append(idx)
            mins.append(comp._norm_min)
            maxs.append(comp._norm_max)
            enhs.append(enh)
        out[f"{tag}_params"] = P
        out[f"{tag}_frames"] = np.stack(frames)
        out[f"{tag}_idx"] = np.stack(idxs)
        out[f"{tag}_min"] = np.array(mins, dtype=np.float32)
        out[f"{tag}_max"] = np.array(maxs, dtype=np.float32)
        comp = MPEGAICompressorImpl()
        comp._normalize_for_compression(enhs[0])
        out[f"{tag}_denorm0"] = comp._denormalize_from_compression(frames[0])
    comp = MPEGAICompressorImpl()
    out["const_frame"] = comp._normalize_for_compression(np.full((5, 4), 2.5, dtype=np.float32))
    # dimension table (core/dimension_calculator.py:36-61, tests/test_dimension_calculator.py:224-238)
    dc = PowerOf4DimensionCalculator()
    sizes = np.array([1, 3, 4, 5, 16, 17, 64, 100, 256, 384, 768, 1024, 1536, 3000, 4096, 10000, 16384,
                      16385, 70000], dtype=np.int64)
    out["dim_sizes"] = sizes
    out["dim_n"] = np.array([dc.calculate_optimal_dimensions(int(s))[0] for s in sizes], dtype=np.int64)
    errs = []
    for s in sizes:
        n = dc.calculate_optimal_dimensions(int(s))
        try:
            dc.calculate_padding_strategy(int(s), n)
            errs.append("")
        except ValueError as e:
            errs.append(str(e))
    out["dim_err"] = np.array(errs)
    return out


def search_fixtures(hq):
    from hilbert_quantization.core.hilbert_mapper import HilbertCurveMapper
    from hilbert_quantization.core.streaming_index_builder import StreamingHilbertIndexGenerator
    from hilbert_quantization.core.search_engine import ProgressiveSimilaritySearchEngine
    from hilbert_quantization.models import QuantizedModel, ModelMetadata
    m = HilbertCurveMapper()
    sg = StreamingHilbertIndexGenerator()
    out = {}
    rng = np.random.default_rng(2024)
    for tag, n, N in [("L64", 64, 160), ("L32", 32, 96)]:
        C = np.zeros((N, n), dtype=np.float64)
        for i in range(N):
            p = rng.standard_normal(n * n if n == 32 else 1536).astype(np.float32)
            pp = np.zeros(n * n, np.float32)
            pp[: len(p)] = p
            C[i] = sg.generate_optimized_indices(m.map_to_2d(pp, (n, n)), n)
        # degenerate rows (SURVEY.md §8a hazards 5/6): zeros, constant 0.1 (np.std != 0), exact
        # constants, duplicates, negations, a constant level-0 segment.
        C[1] = 0.0
        C[2] = 0.1
        C[3] = 0.5
        C[4] = C[10]
        C[5] = -C[11]
        C[6, : n // 2] = 0.25
        C[7] = C[10]
        C[8] = C[12] * 2.0 + 1.0
        Q = np.stack([C[10] + rng.normal(0, 0.01, n), C[20].copy(), np.full(n, 0.5), rng.standard_normal(n),
                      C[2].copy(), C[6].copy()])
        eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=20)
        levels = eng._parse_index_structure(Q[0], n)
        nl = len(levels)
        per = np.zeros((len(Q), N, nl))
        for a in range(len(Q)):
            for b in range(N):
                for lv in range(nl):
                    per[a, b, lv] = eng.compare_indices_at_level(Q[a], C[b], lv)
        ov = np.zeros((len(Q), N))
        for a in range(len(Q)):
            for b in range(N):
                ov[a, b] = eng._calculate_overall_similarity(Q[a], C[b])[0]
        models = []
        for b in range(N):
            md = ModelMetadata(model_name=f"m{b}", original_size_bytes=1, compressed_size_bytes=1,
                               compression_ratio=1.0, quantization_timestamp="t")
            models.append(QuantizedModel(compressed_data=b"x", original_dimensions=(n, n), parameter_count=1,
                                         compression_quality=0.8, hierarchical_indices=C[b], metadata=md))
        K = 10
        bf_ids = np.full((len(Q), K), -1, np.int64)
        bf_sc = np.zeros((len(Q), K))
        pg_ids = np.full((len(Q), K), -1, np.int64)
        pg_sc = np.zeros((len(Q), K))
        pg_err = np.zeros((len(Q), K))
        for a in range(len(Q)):
            r = eng.brute_force_search(Q[a], models, K)
            for j, x in enumerate(r):
                bf_ids[a, j] = int(x.model.model_id[1:])
                bf_sc[a, j] = x.similarity_score
            r = eng.progressive_search(Q[a], models, K)
            for j, x in enumerate(r):
                pg_ids[a, j] = int(x.model.model_id[1:])
                pg_sc[a, j] = x.similarity_score
                pg_err[a, j] = x.reconstruction_error
        # threshold-fallback case: every candidate scores below 0.1 -> first argmax survives
        negC = -np.tile(Q[3], (30, 1)) * (1.0 + 0.01 * np.arange(30)[:, None])
        negmodels = []
        for b in range(30):
            md = ModelMetadata(model_name=f"m{b}", original_size_bytes=1, compressed_size_bytes=1,
                               compression_ratio=1.0, quantization_timestamp="t")
            negmodels.append(QuantizedModel(compressed_data=b"x", original_dimensions=(n, n), parameter_count=1,
                                            compression_quality=0.8, hierarchical_indices=negC[b], metadata=md))
        r = eng.progressive_search(Q[3], negmodels, K)
        out[f"{tag}_fallback_C"] = negC
        out[f"{tag}_fallback_ids"] = np.array([int(x.model.model_id[1:]) for x in r], dtype=np.int64)
        out[f"{tag}_fallback_sc"] = np.array([x.similarity_score for x in r])
        out[f"{tag}_C"] = C
        out[f"{tag}_Q"] = Q
        out[f"{tag}_per_level"] = per
        out[f"{tag}_overall"] = ov
        out[f"{tag}_bf_ids"] = bf_ids
        out[f"{tag}_bf_sc"] = bf_sc
        out[f"{tag}_pg_ids"] = pg_ids
        out[f"{tag}_pg_sc"] = pg_sc
        out[f"{tag}_pg_err"] = pg_err
    struct = []
    for L in list(range(1, 130)) + [256, 1024, 4096]:
        for lv in ProgressiveSimilaritySearchEngine()._parse_index_structure(np.zeros(L), L):
            struct.append((L, lv.grid_size, lv.start_index, lv.end_index, int(lv.is_offset_sampling)))
    out["parse_struct"] = np.array(struct, dtype=np.int64)
    return out


def _f32_rows(rng, L, N):
    """float32 index vectors: random rows plus every case where NumPy's float32 statistics leave the
    f64 model (SURVEY.md §8a hazard 5): inexact constants, 1-ulp near-constants, f32
    underflow of d*d, tiny / huge magnitudes, a large mean / std ratio."""
    C = rng.standard_normal((N, L)).astype(np.float32)
    C[1] = np.float32(0.1)
    C[2] = np.float32(1.7)
    C[3] = 0.0
    C[4] = np.float32(0.5)
    C[5, : L // 2] = np.float32(0.1)
    C[6] = C[1]
    v = np.float32(1.7)
    C[7] = v
    C[7, [3, 9, 17]] = np.nextafter(v, np.float32(2))          # 1-ulp near-constant
    C[8] = np.float32(0.1)
    C[8, ::5] = np.nextafter(np.float32(0.1), np.float32(1))
    C[9] = np.where(np.arange(L) % 2 == 0, np.float32(1e-25), np.float32(2e-25))  # d*d underflows
    C[10] = (rng.standard_normal(L) * 1e-20).astype(np.float32)  # squares in the f32 denormal range
    C[11] = (1000.0 + rng.standard_normal(L) * 1e-3).astype(np.float32)  # large mean / std ratio
    C[12] = C[11] + np.float32(0.001)
    C[13] = -C[20]
    C[14] = C[20] * np.float32(2.0) + np.float32(1.0)
    C[15] = C[7]
    C[15, 0] = np.nextafter(v, np.float32(0))
    return C


def search_f32_fixtures(hq):
    """compare_indices_at_level / _calculate_overall_similarity / searches on float32 index vectors,
    run by the reference itself: NumPy keeps the array dtype, so np.std, the normalisation and (when
    both arrays are float32) the whole score run in float32, and the score is a numpy.float32 unless a
    constant branch or a clamp returns a Python float (core/search_engine.py:111-230).  Also a float64
    query against float32 candidates (mixed) and a pool mixing both dtypes."""
    from hilbert_quantization.core.search_engine import ProgressiveSimilaritySearchEngine
    from hilbert_quantization.models import QuantizedModel, ModelMetadata
    out = {}
    rng = np.random.default_rng(4242)

    def models_of(rows):
        ms = []
        for b, r in enumerate(rows):
            md = ModelMetadata(model_name=f"m{b}", original_size_bytes=1, compressed_size_bytes=1,
                               compression_ratio=1.0, quantization_timestamp="t")
            ms.append(QuantizedModel(compressed_data=b"x", original_dimensions=(8, 8), parameter_count=1,
                                     compression_quality=0.8, hierarchical_indices=r, metadata=md))
        return ms

    for tag, L, N in [("L64", 64, 72), ("L32", 32, 48), ("L256", 256, 40)]:
        C = _f32_rows(rng, L, N)
        Q = np.stack([C[20] + rng.normal(0, 0.01, L).astype(np.float32), C[1], C[7], C[8], C[9], C[10], C[11],
                      C[3], rng.standard_normal(L).astype(np.float32)])
        eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=20)
        nl = len(eng._parse_index_structure(Q[0], L))
        for qtag, QQ in [("q32", Q), ("q64", Q.astype(np.float64))]:
            per = np.zeros((len(QQ), N, nl))
            per_t = np.zeros((len(QQ), N, nl), np.int8)
            ov = np.zeros((len(QQ), N))
            ov_t = np.zeros((len(QQ), N), np.int8)
            for a in range(len(QQ)):
                for b in range(N):
                    for lv in range(nl):
                        v = eng.compare_indices_at_level(QQ[a], C[b], lv)
                        per[a, b, lv] = float(v)
                        per_t[a, b, lv] = isinstance(v, np.float32)
                    v = eng._calculate_overall_similarity(QQ[a], C[b])[0]
                    ov[a, b] = float(v)
                    ov_t[a, b] = isinstance(v, np.float32)
            out[f"{tag}_{qtag}_per_level"] = per
            out[f"{tag}_{qtag}_per_level_f32"] = per_t
            out[f"{tag}_{qtag}_overall"] = ov
            out[f"{tag}_{qtag}_overall_f32"] = ov_t
        # searches: float32 pool, and a pool mixing float32 / float64 rows (odd rows widened)
        pools = {"pool32": [C[b] for b in range(N)],
                 "poolmix": [C[b] if b % 2 == 0 else C[b].astype(np.float64) for b in range(N)]}
        K = 10
        for ptag, rows in pools.items():
            models = models_of(rows)
            for stag, fn in [("bf", eng.brute_force_search), ("pg", eng.progressive_search)]:
                ids = np.full((len(Q), K), -1, np.int64)
                sc = np.zeros((len(Q), K))
                for a in range(len(Q)):
                    for j, x in enumerate(fn(Q[a], models, K)):
                        ids[a, j] = int(x.model.model_id[1:])
                        sc[a, j] = float(x.similarity_score)
                out[f"{tag}_{ptag}_{stag}_ids"] = ids
                out[f"{tag}_{ptag}_{stag}_sc"] = sc
        out[f"{tag}_C"] = C
        out[f"{tag}_Q"] = Q
        if tag == "L64":
            out.update(_threshold_rounding_fixtures(eng, models_of, pools, Q, N))
    return out


def _threshold_rounding_fixtures(eng, models_of, pools, Q, N):
    """the reference compares a numpy.float32 level score with the Python-float threshold in
    float32 (NumPy 2, NEP 50: the threshold is rounded to float32), a Python-float score in float64.  Per
    query, s = the second-best float32-typed level-0 score over the pool; thresholds a quarter ulp above
    (progressive, `>=`, core/search_engine.py:284-292) and below (the video engine's level-0 frame scan,
    `>`, core/video_search.py:236-264) round to s in float32, so the reference keeps / drops s where a
    float64 comparison would not.  Pools: float32 and mixed float32 / float64 rows, each with ("full") and
    without ("safe": the scan path) the float32-unsafe rows 3 (all zero), 9 and 10.  Thresholds are Python floats (as a caller passes them;
    a numpy float64 threshold would compare in float64)."""
    from hilbert_quantization.core.search_engine import ProgressiveSimilaritySearchEngine
    out = {}
    keep = [b for b in range(N) if b not in (3, 9, 10)]
    for ptag, rows_all in pools.items():
        for sub, idxs in (("full", list(range(N))), ("safe", keep)):
            rows = [rows_all[b] for b in idxs]
            models = models_of(rows)
            K = 10
            t_ge, t_gt = np.zeros(len(Q)), np.zeros(len(Q))
            pg_ids, fr_ids = np.full((len(Q), K), -1, np.int64), np.full((len(Q), K), -1, np.int64)
            pg_sc, fr_sc = np.zeros((len(Q), K)), np.zeros((len(Q), K))
            for a in range(len(Q)):
                s0 = [eng.compare_indices_at_level(Q[a], r, 0) for r in rows]
                typed = sorted({float(v) for v in s0 if isinstance(v, np.float32)}, reverse=True)
                if typed:  # (a constant query has no float32-typed score: the plain threshold 0.1)
                    s = np.float32(typed[1] if len(typed) > 1 else typed[0])
                    up = float(np.nextafter(s, np.float32(2)) - s)
                    down = float(s - np.nextafter(s, np.float32(-2)))
                    t_ge[a], t_gt[a] = float(s) + up / 4, float(s) - down / 4
                    assert np.float32(t_ge[a]) == s and np.float32(t_gt[a]) == s
                else:
                    t_ge[a] = t_gt[a] = 0.1
                e2 = ProgressiveSimilaritySearchEngine(similarity_threshold=float(t_ge[a]), max_candidates_per_level=20)
                for j, x in enumerate(e2.progressive_search(Q[a], models, K)):
                    pg_ids[a, j] = int(x.model.model_id[1:])
                    pg_sc[a, j] = float(x.similarity_score)
                # VideoEnhancedSearchEngine._hierarchical_search (video_search.py:236-264) over the pool's
                # index vectors: level-0 similarity > threshold, stable sort desc, top K
                hits = [(v, b) for b, v in enumerate(s0) if v > float(t_gt[a])]
                hits.sort(key=lambda h: h[0], reverse=True)
                for j, (v, b) in enumerate(hits[:K]):
                    fr_ids[a, j] = b
                    fr_sc[a, j] = float(v)
            key = f"thr_{ptag}_{sub}"
            out[f"{key}_t_ge"], out[f"{key}_t_gt"] = t_ge, t_gt
            out[f"{key}_pg_ids"], out[f"{key}_pg_sc"] = pg_ids, pg_sc
            out[f"{key}_fr_ids"], out[f"{key}_fr_sc"] = fr_ids, fr_sc
            out[f"{key}_rows"] = np.array(idxs, np.int64)
    return out


def rag_score_fixtures(hq):
    from hilbert_quantization.rag.search import engine as E
    cls = E.RAGSearchEngineImpl if hasattr(E, "RAGSearchEngineImpl") else None
    if cls is None:
        cands = [v for v in vars(E).values() if isinstance(v, type) and hasattr(v, "_compare_multi_level_indices")]
        cls = cands[0]
    obj = cls.__new__(cls)  # scoring helpers use no instance state beyond each other
    rng = np.random.default_rng(5)
    out = {}
    A = rng.standard_normal((8, 32, 32)).astype(np.float32)
    A[3] = 0.0
    B = A[0] + rng.normal(0, 0.3, (32, 32)).astype(np.float32)
    out["cos_A"] = A
    out["cos_B"] = B
    out["cos"] = np.array([obj._calculate_embedding_cosine_similarity(B, A[i]) for i in range(8)])
    ML = rng.standard_normal((6, 3, 64))
    out["ml_C"] = ML
    out["ml_Q"] = ML[0] + rng.normal(0, 0.2, (3, 64))
    out["ml"] = np.array([obj._compare_multi_level_indices(out["ml_Q"], ML[i]) for i in range(6)])
    out["ml_w3"] = obj._calculate_granularity_weights(3)
    out["ml_w5"] = obj._calculate_granularity_weights(5)
    # spatial locality (engine.py:662-714) on enhanced images (the RAG generator's index rows appended):
    # heights detected per image (engine.py:134-162, 604-620), float32 and float64 inputs
    from hilbert_quantization.rag.embedding_generation.hierarchical_index_generator import (
        HierarchicalIndexGenerator as RagGen)
    rg = RagGen()
    for tag, n, dt in (("s64f", 64, np.float32), ("s64d", 64, np.float64), ("s32f", 32, np.float32),
                       ("s8d", 8, np.float64)):
        base = rng.standard_normal((n, n)).astype(dt)
        imgs = [base, base + rng.normal(0, 0.3, (n, n)).astype(dt), rng.standard_normal((n, n)).astype(dt),
                -base, np.zeros((n, n), dt), base * 3.0 + 1.0]
        short = base.copy()
        short[n - 1, : (3 * n) // 4] = 0.0          # last data row mostly zeros: a different detected height
        imgs.append(short)
        enh = np.stack([np.asarray(rg.generate_multi_level_indices(im)).astype(dt) for im in imgs])
        out[f"{tag}_enh"] = enh
        out[f"{tag}_heights"] = np.array([obj._detect_original_embedding_height(e) for e in enh], dtype=np.int64)
        out[f"{tag}_spatial"] = np.array([[float(obj._calculate_spatial_locality_similarity(enh[a], enh[b]))
                                           for b in range(len(enh))] for a in range(2)])
    tiny = rng.standard_normal((2, 5, 4))                  # ws < 2: one cosine over the block
    out["tiny_enh"] = tiny
    out["tiny_spatial"] = np.array([float(obj._calculate_spatial_locality_similarity(tiny[0], tiny[1]))])
    # progressive threshold (engine.py:243-287): levels 0..4, candidate lists in arbitrary id order
    sc = np.round(rng.uniform(0.0, 1.0, 200), 3)
    sc[:5] = [0.6000000000000001, 0.6, 0.5, 0.3, 0.8]     # on the level thresholds (Python float sums)
    ids = rng.permutation(1000)[:200]
    out["thr_scores"], out["thr_ids"] = sc, ids
    for level in range(5):
        for cut in (200, 37, 1):
            got = obj._apply_progressive_threshold(list(zip(ids[:cut].tolist(), sc[:cut].tolist())), level)
            out[f"thr_l{level}_n{cut}"] = np.array(got + [-1] * (200 - len(got)), dtype=np.int64)
    return out


def precomputed_fixtures(hq):
    """core/precomputed_hilbert_index.py: overlapping-square averages and the f32 level similarity."""
    import contextlib
    import io
    from hilbert_quantization.core.precomputed_hilbert_index import (
        PrecomputedHilbertIndexer, PrecomputedSimilaritySearchEngine)
    from hilbert_quantization.core.hilbert_mapper import HilbertCurveMapper
    rng = np.random.default_rng(77)
    out = {}
    ix = PrecomputedHilbertIndexer()
    imgs = {}
    for n in [2, 4, 8, 16, 32, 64, 128]:
        imgs[f"n{n}"] = (rng.standard_normal((n, n)) * rng.uniform(0.1, 3)).astype(np.float32)
    p = rng.standard_normal(1536).astype(np.float32)
    padded = np.zeros(4096, dtype=np.float32)
    padded[:1536] = p
    imgs["pad1536"] = HilbertCurveMapper().map_to_2d(padded, (64, 64))
    imgs["const32"] = np.full((32, 32), 0.25, dtype=np.float32)
    imgs["f64_16"] = rng.standard_normal((16, 16))
    for name, img in imgs.items():
        with contextlib.redirect_stdout(io.StringIO()):
            idx = ix.create_precomputed_index(img, name)
        out[f"img_{name}"] = img
        out[f"avg_{name}"] = np.concatenate([lv.averages for lv in idx.levels])
        out[f"meta_{name}"] = np.array([[lv.grid_size, lv.square_size, lv.num_squares] for lv in idx.levels],
                                       dtype=np.int64)
        out[f"xy_{name}"] = np.array([xy for lv in idx.levels for xy in lv.square_coordinates], dtype=np.int64)
        out[f"bytes_{name}"] = np.array(idx.total_storage_bytes, dtype=np.int64)
    # similarity: query 64x64 image against noisy copies, a constant image, a negated image
    eng = PrecomputedSimilaritySearchEngine(ix)
    base = imgs["pad1536"]
    cands = [base, base + rng.normal(0, 0.05, base.shape).astype(np.float32),
             base + rng.normal(0, 0.5, base.shape).astype(np.float32), -base,
             np.full((64, 64), 0.1, dtype=np.float32), rng.standard_normal((64, 64)).astype(np.float32),
             base * 2.0 + 1.0, np.zeros((64, 64), dtype=np.float32)]
    with contextlib.redirect_stdout(io.StringIO()):
        qi = ix.create_precomputed_index(base, "q")
        cis = [ix.create_precomputed_index(c.astype(np.float32), f"c{i}") for i, c in enumerate(cands)]
    out["sim_cands"] = np.stack([c.astype(np.float32) for c in cands])
    sims, types, lev = [], [], []
    for ci in cis:
        v = eng._calculate_precomputed_similarity(qi, ci)
        sims.append(float(v))
        types.append(0 if isinstance(v, np.floating) and v.dtype == np.float32 else 1)
        lev.append([float(eng._compare_precomputed_levels(a, b)) for a, b in zip(qi.levels, ci.levels)])
    out["sim_overall"] = np.array(sims)
    out["sim_type"] = np.array(types, dtype=np.int64)
    out["sim_levels"] = np.array(lev)
    # constant-vs-constant level branch within 1e-6 (float32 comparison) and the 0.1 branch
    a = np.full(5, 0.5, dtype=np.float32)
    out["lvl_const_pairs"] = np.array([0.5, 0.5000005, 0.500001, 0.6], dtype=np.float32)
    from hilbert_quantization.core.precomputed_hilbert_index import PrecomputedLevel
    lv = lambda arr: PrecomputedLevel(2, 2, len(arr), arr, [])  # noqa: E731
    out["lvl_const_vals"] = np.array([float(eng._compare_precomputed_levels(lv(a), lv(np.full(5, v, dtype=np.float32))))
                                      for v in out["lvl_const_pairs"]])
    return out


def store_fixtures(hq):
    """Storage metadata written by the reference's own savers, kept as the JSON text
    they produced (data), plus the reference's own reading of it:
    * core/video_storage.py:579-631 `_save_video_metadata` (+ `_save_global_index`) for three videos of 40
      frames (duplicates across videos), read back by `_load_existing_index` (:633-691); the level-0
      similarity of every (query, frame) pair by the reference's compare_indices_at_level, keyed by model
      id (the visiting order is the directory's glob order, so the ranking is rebuilt where the files lie);
    * rag/video_storage/dual_storage.py:86-121 `_save_metadata` for 12 frames, read back by
      `_load_existing_metadata` (:51-84)."""
    import tempfile
    from pathlib import Path
    from hilbert_quantization.core import video_storage as VS
    from hilbert_quantization.core.search_engine import ProgressiveSimilaritySearchEngine
    from hilbert_quantization.models import ModelMetadata
    rng = np.random.default_rng(6)
    C = rng.standard_normal((3 * 40, 64)).cumsum(1) * 0.1
    C[45] = C[3]
    C[90] = C[3]
    out = {}
    with tempfile.TemporaryDirectory() as d:
        st = VS.VideoModelStorage.__new__(VS.VideoModelStorage)
        st.storage_dir = Path(d)
        st._global_index_path = Path(d) / "video_index.json"
        st._video_index, st._model_to_video_map = {}, {}
        st._video_file_counter, st.max_frames_per_video, st.frame_rate, st.video_codec = 3, 1000, 30.0, "mp4v"
        for v in range(3):
            frames = []
            for i in range(40):
                md = ModelMetadata(model_name=f"m{40 * v + i}", original_size_bytes=6144, compressed_size_bytes=900,
                                   compression_ratio=6144 / 900, quantization_timestamp="2025-09-05 12:00:00",
                                   model_architecture="mlp" if i % 2 else None, additional_info={"layer": i})
                frames.append(VS.VideoFrameMetadata(
                    frame_index=i, model_id=f"m{40 * v + i}", original_parameter_count=1536, compression_quality=0.8,
                    hierarchical_indices=C[40 * v + i], model_metadata=md, frame_timestamp=1000.0 + i,
                    similarity_features=rng.standard_normal(4) if i % 7 == 0 else None))
            vm = VS.VideoStorageMetadata(video_path=str(Path(d) / f"video_{v}.mp4"), total_frames=40, frame_rate=30.0,
                                         video_codec="mp4v", frame_dimensions=(65, 64),
                                         creation_timestamp="2025-09-05 12:00:00", total_models_stored=40,
                                         average_compression_ratio=6.8, frame_metadata=frames)
            st._video_index[vm.video_path] = vm
            st._save_video_metadata(vm)
        names = sorted(p.name for p in Path(d).glob("*.json"))
        out["video_json_names"] = np.array(names)
        out["video_json_texts"] = np.array([(Path(d) / n).read_text().replace(d, "@STORE@") for n in names])
        st2 = VS.VideoModelStorage.__new__(VS.VideoModelStorage)
        st2.storage_dir, st2._video_index, st2._model_to_video_map = Path(d), {}, {}
        st2._load_existing_index()
        loaded = {fm.model_id: fm for vm in st2._video_index.values() for fm in vm.frame_metadata}
        ids = sorted(loaded, key=lambda s: int(s[1:]))
        out["video_loaded_ids"] = np.array(ids)
        out["video_loaded_idx"] = np.stack([np.asarray(loaded[m].hierarchical_indices) for m in ids])
        out["video_loaded_map"] = np.array([[int(st2._model_to_video_map[m][0].rsplit("video_", 1)[1][0]),
                                             st2._model_to_video_map[m][1]] for m in ids])
        eng = ProgressiveSimilaritySearchEngine()
        Q = np.concatenate([C[[3, 50, 100]], C[[7, 60]] + rng.normal(0, 0.05, (2, 64))])
        out["video_queries"] = Q
        out["video_sims"] = np.array([[float(eng.compare_indices_at_level(q, loaded[m].hierarchical_indices, 0))
                                       for m in ids] for q in Q])
    # RAG dual storage
    from hilbert_quantization.rag.video_storage import dual_storage as DS
    from hilbert_quantization.rag.models import DocumentChunk, VideoFrameMetadata as RVF
    with tempfile.TemporaryDirectory() as d:
        ds = DS.DualVideoStorageImpl.__new__(DS.DualVideoStorageImpl)
        ds.metadata_dir = d
        ds.current_video_index, ds.current_frame_count = 1, 12
        ds.frame_metadata = []
        for i in range(12):
            ch = DocumentChunk(content=f"chunk {i} text " * (i + 1), ipfs_hash=f"Qm{i:044d}", source_path=f"doc{i % 3}.txt",
                               start_position=100 * i, end_position=100 * i + 50 + i, chunk_sequence=i,
                               creation_timestamp="2025-09-05T12:00:00", chunk_size=50 + i)
            ds.frame_metadata.append(RVF(frame_index=i, chunk_id=f"c{i}", ipfs_hash=ch.ipfs_hash,
                                         source_document=ch.source_path, compression_quality=0.8,
                                         hierarchical_indices=[], embedding_model="all-MiniLM-L6-v2",
                                         frame_timestamp=2000.0 + i, chunk_metadata=ch))
        ds._save_metadata()
        text = Path(d, "dual_video_metadata.json").read_text()
        out["dual_json_text"] = np.array(text)
        ds2 = DS.DualVideoStorageImpl.__new__(DS.DualVideoStorageImpl)
        ds2.metadata_dir, ds2.current_video_index, ds2.current_frame_count, ds2.frame_metadata = d, 0, 0, []
        ds2._load_existing_metadata()
        out["dual_state"] = np.array([ds2.current_video_index, ds2.current_frame_count])
        out["dual_loaded"] = np.array([[str(f.frame_index), f.chunk_id, f.ipfs_hash, f.source_document,
                                        repr(f.compression_quality), f.embedding_model, repr(f.frame_timestamp),
                                        f.chunk_metadata.content, str(f.chunk_metadata.chunk_size)]
                                       for f in ds2.frame_metadata])
    return out


def api_fixtures(hq):
    """End-to-end HilbertQuantizer (api.py:120-297, core/pipeline.py:71-233, core/compressor.py:43-148):
    quantize 8 seeded vectors per length with the pre-computed index on, reconstruct each in order (the
    compressor's instance state: every decompress de-normalises with the LAST compress's min / max),
    then search the 8 models with 4 queries (each query is itself quantized first, api.py:268)."""
    import contextlib
    import io
    from hilbert_quantization.api import HilbertQuantizer
    rng = np.random.default_rng(4242)
    out = {}
    try:  # 1536 values on 64 x 64 = efficiency 0.375 < the default minimum 0.5: the reference refuses
        HilbertQuantizer(use_precomputed_indexing=True).quantize(rng.standard_normal(1536).astype(np.float32),
                                                                 model_id="eff")
        out["d1536_error"] = np.array("")
    except Exception as e:  # noqa: BLE001
        out["d1536_error"] = np.array(f"{type(e).__name__}: {e}")
    for d in (1024, 3000, 4096):
        tag = f"d{d}"
        hqz = HilbertQuantizer(use_precomputed_indexing=True)
        P = rng.standard_normal((8, d)).astype(np.float32)
        P[5] = P[2] * 0.5 + 0.01            # a near-duplicate direction
        P[7] = P[3]                          # an exact duplicate: tie order follows the pool
        out[f"{tag}_params"] = P
        with contextlib.redirect_stdout(io.StringIO()):
            models = [hqz.quantize(P[i], model_id=f"{tag}_m{i}") for i in range(8)]
            for i, m in enumerate(models):
                out[f"{tag}_payload_{i}"] = np.frombuffer(m.compressed_data, dtype=np.uint8).copy()
                out[f"{tag}_hidx_{i}"] = np.asarray(m.hierarchical_indices)
            out[f"{tag}_dims"] = np.array([m.original_dimensions for m in models], dtype=np.int64)
            out[f"{tag}_count"] = np.array([m.parameter_count for m in models], dtype=np.int64)
            out[f"{tag}_quality"] = np.array([m.compression_quality for m in models])
            comp = hqz.quantization_pipeline.compressor
            out[f"{tag}_minmax_last"] = np.array([comp._norm_min, comp._norm_max], dtype=np.float64) \
                if hasattr(comp, "_norm_min") else np.zeros(0)
            out[f"{tag}_recon"] = np.stack([np.asarray(hqz.reconstruct(m), dtype=np.float32) for m in models])
            Qs = np.stack([P[2] + rng.normal(0, 0.05, d).astype(np.float32), P[3] + 0.0,
                           rng.standard_normal(d).astype(np.float32), P[6] * 2.0]).astype(np.float32)
            out[f"{tag}_queries"] = Qs
            ids = np.full((4, 8), -1, dtype=np.int64)
            sc = np.zeros((4, 8))
            err = np.zeros((4, 8))
            for a in range(4):
                r = hqz.search(Qs[a], candidate_models=models, max_results=8)
                for j, x in enumerate(r):
                    ids[a, j] = int(x.model.metadata.model_name.rsplit("_m", 1)[1])
                    sc[a, j] = x.similarity_score
                    err[a, j] = x.reconstruction_error
            out[f"{tag}_search_ids"], out[f"{tag}_search_sc"], out[f"{tag}_search_err"] = ids, sc, err
    return out


def _craft_search(score_fn, target_fn, seed, want=1):
    """Inputs for the float32 / Python-float sort-key goldens: a float32 query q and candidates
    c(t) = mu + a (q - mean q) + t d along which a float32 score crosses target_fn(q); every float32 t
    around the crossing is tried until the score equals the target exactly.  The oracle only steers the
    search; the fixture's outputs are the reference's."""
    rng = np.random.default_rng(seed)
    found = []
    for _ in range(400):
        mu = rng.uniform(0.6, 1.4)
        q = (rng.standard_normal(64) + mu).astype(np.float32)
        d1 = rng.standard_normal(64).astype(np.float32)
        a = rng.uniform(-1.3, -0.7)
        base = (mu + a * (q - q.mean())).astype(np.float32)
        target = target_fn(q)
        if target is None:
            continue
        ts = np.linspace(0, 2, 2001).astype(np.float32)
        sc = score_fn(q, (base[None, :] + ts[:, None] * d1[None, :]).astype(np.float32))
        for i in np.nonzero((sc[:-1] - target) * (sc[1:] - target) <= 0)[0][:3]:
            lo, hi = ts[i].view(np.int32), ts[i + 1].view(np.int32)
            tt = np.arange(lo, hi + 1, dtype=np.int32).view(np.float32)
            cc = (base[None, :] + tt[:, None] * d1[None, :]).astype(np.float32)
            hit = np.nonzero(score_fn(q, cc) == target)[0]
            if len(hit):
                found.append((q, cc[hit[0]]))
                break
        if len(found) >= want:
            return found
    raise RuntimeError("no crafted pair found")


def sortkey_fixtures(hq):
    """Python's mixed-type sort keys (core/search_engine.py:291 and :386, NumPy 2 / NEP 50): a numpy
    float32 score compares with a Python-float score in float32, so float32(0.1) ties the Python 0.1 of
    the one-constant-side branch (level-0 filter sort) and an all-constant-branch Python-float overall ties
    the float32 overall equal to its float32 rounding (final sort); ties keep the pool / survivor order."""
    import contextlib
    import io
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import hq_oracle as O
    from hilbert_quantization.core.search_engine import ProgressiveSimilaritySearchEngine
    from hilbert_quantization.models import ModelMetadata, QuantizedModel
    out = {}

    def pool_of(rows):
        return [QuantizedModel(b"x", (8, 8), 1, 0.8, np.asarray(r, dtype=np.float32),
                               ModelMetadata(f"m{i}", 1, 1, 1.0, "t")) for i, r in enumerate(rows)]

    def run(tag, q, rows, M, K):
        eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=M)
        pool = pool_of(rows)
        with contextlib.redirect_stdout(io.StringIO()):
            r = eng.progressive_search(np.asarray(q, dtype=np.float32), pool, K)
            b = eng.brute_force_search(np.asarray(q, dtype=np.float32), pool, K)
        out[f"{tag}_q"] = np.asarray(q, dtype=np.float32)
        out[f"{tag}_C"] = np.stack(rows).astype(np.float32)
        out[f"{tag}_M"] = np.array(M)
        out[f"{tag}_pg_ids"] = np.array([int(x.model.model_id[1:]) for x in r], dtype=np.int64)
        out[f"{tag}_pg_sc"] = np.array([float(x.similarity_score) for x in r])
        out[f"{tag}_pg_f32"] = np.array([isinstance(x.similarity_score, np.float32) for x in r])
        out[f"{tag}_bf_ids"] = np.array([int(x.model.model_id[1:]) for x in b], dtype=np.int64)
        out[f"{tag}_bf_sc"] = np.array([float(x.similarity_score) for x in b])
        out[f"{tag}_lv0"] = np.array([float(eng.compare_indices_at_level(q, c, 0)) for c in rows])
        out[f"{tag}_lv0_f32"] = np.array([isinstance(eng.compare_indices_at_level(q, c, 0), np.float32) for c in rows])

    # (1) level-0 filter: a float32 score exactly float32(0.1) against the Python 0.1 of a constant level-0
    # segment; M keeps exactly one of the two after the candidates scoring above them
    t01 = float(np.float32(0.1))
    [(q, cF)] = _craft_search(lambda q, C: O.level_similarity(q, C, 0), lambda q: t01, 13)
    rng = np.random.default_rng(31)
    high = [(q + rng.normal(0, 0.05 * (i + 1), 64)).astype(np.float32) for i in range(6)]
    cP = rng.standard_normal(64).astype(np.float32)
    cP[:32] = np.float32(2.5)                     # constant level-0 segment: the reference returns 0.1
    low = [(-q + rng.normal(0, 0.01, 64)).astype(np.float32) for _ in range(5)]
    run("lv0_PF", q, high + [cP, cF] + low, 7, 7)   # Python 0.1 first in the pool: it survives (tie)
    run("lv0_FP", q, high + [cF, cP] + low, 7, 7)   # float32 0.1 first: it survives

    # (2) final sort: an all-constant-branch Python-float overall against the float32 overall equal to its
    # float32 rounding
    def p_overall(q):
        cc = np.full(64, np.float32(q[43] + 0.5), dtype=np.float32)
        P = O.overall_similarity(q, cc[None])[0][0]
        return float(np.float32(P)) if float(np.float32(P)) != P else None

    [(q2, cF2)] = _craft_search(lambda q, C: O.overall_similarity(q, C)[0], p_overall, 17)
    cP2 = np.full(64, np.float32(q2[43] + 0.5), dtype=np.float32)
    rng = np.random.default_rng(37)
    other = [(q2 + rng.normal(0, 0.3 * (i + 1), 64)).astype(np.float32) for i in range(4)]
    run("ov_PF", q2, other[:2] + [cP2, cF2] + other[2:], 20, 6)
    run("ov_FP", q2, other[:2] + [cF2, cP2] + other[2:], 20, 6)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated fixture names to (re)generate")
    a = ap.parse_args()
    hq = _import_reference(a.ref)
    only = set(filter(None, a.only.split(",")))
    for name, fn in [("mapper", mapper_fixtures), ("index", index_fixtures), ("quant", quant_fixtures),
                     ("search", search_fixtures), ("search_f32", search_f32_fixtures),
                     ("rag_score", rag_score_fixtures), ("stores", store_fixtures),
                     ("precomputed", precomputed_fixtures), ("api", api_fixtures),
                     ("sortkey", sortkey_fixtures)]:
        if only and name not in only:
            continue
        d = fn(hq)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"wrote {path}: {len(d)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
