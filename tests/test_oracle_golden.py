"""Pin the CPU oracle (oracle/hq_oracle.py) to the reference: golden vectors generated from the real
reference (tests/golden/make_golden.py) and the reference's own known-answer tests.
CPU only."""
import math

import numpy as np
import pytest

from oracle import hq_oracle as O

# ---------------------------------------------------------------- NumPy-order reductions


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_np_order_sum_mean_std(dtype):
    rng = np.random.default_rng(3)
    for n in list(range(1, 140)) + [255, 256, 300, 1024]:
        X = (rng.standard_normal((7, n)) * 10 ** rng.uniform(-3, 3)).astype(dtype)
        s = O.np_sum_rows(X)
        m = O.np_mean_rows(X)
        sd = O.np_std_rows(X)
        for i in range(7):
            assert s[i] == np.add.reduce(X[i])
            assert m[i] == np.mean(X[i])
            assert sd[i] == np.std(X[i])


def test_np_std_constant_point_one():
    # SURVEY.md §8a hazard 5: np.std([0.1]*3) is 1.39e-17, not 0
    x = np.full((1, 3), 0.1)
    assert O.np_std_rows(x)[0] == np.std(x[0]) != 0.0


# ---------------------------------------------------------------- M rows


def test_reference_kats():
    # tests/test_hilbert_mapper.py:23, :43-46; tests/test_rag_hilbert_mapper.py:317
    xs, ys = O.hilbert_table(2)
    assert list(zip(xs, ys)) == [(0, 0), (0, 1), (1, 1), (1, 0)]
    xs, ys = O.hilbert_table(4)
    assert list(zip(xs, ys))[:8] == [(0, 0), (1, 0), (1, 1), (0, 1), (0, 2), (0, 3), (1, 3), (1, 2)]
    # tests/test_hilbert_mapper.py:173-182 and tests/test_rag_hilbert_mapper.py:694-701
    assert list(O.map_from_2d(np.array([[1, 4], [2, 3]]))) == [1, 2, 3, 4]
    assert list(O.map_from_2d(np.array([[1, 2], [3, 4]]))) == [1, 3, 4, 2]
    with pytest.raises(ValueError, match="power of 2"):
        O.hilbert_table(3)


def test_coords_and_xy2d_golden(golden):
    g = golden("mapper")
    for n in [1, 2, 4, 8, 16, 32, 64, 128]:
        xs, ys = O.hilbert_table(n)
        np.testing.assert_array_equal(np.stack([xs, ys], 1), g[f"coords_n{n}"])
    for n in [1, 2, 4, 8, 16, 32, 64]:
        yy, xx = np.mgrid[0:n, 0:n]
        np.testing.assert_array_equal(O.hilbert_xy2d(xx, yy, n), g[f"xy2d_n{n}"])


def test_map_golden(golden):
    g = golden("mapper")
    k = 0
    while f"map_in_{k}" in g:
        p = g[f"map_in_{k}"]
        img = g[f"map_out_{k}"]
        n = img.shape[0]
        out = O.map_to_2d(p, n)
        assert out.dtype == img.dtype
        assert out.tobytes() == img.tobytes()
        assert g[f"rag_map_out_{k}"].tobytes() == img.tobytes()
        un = O.map_from_2d(img)
        assert un.tobytes() == g[f"unmap_out_{k}"].tobytes() == g[f"rag_unmap_out_{k}"].tobytes()
        k += 1
    assert k >= 8


# ---------------------------------------------------------------- S1 / I rows


def test_dimension_table(golden):
    g = golden("quant")
    for s, n, err in zip(g["dim_sizes"], g["dim_n"], g["dim_err"]):
        assert O.optimal_dimensions(int(s)) == (n, n)
        if err:
            with pytest.raises(ValueError) as e:
                O.check_efficiency(int(s), (n, n))
            assert str(e.value) == str(err)
        else:
            O.check_efficiency(int(s), (n, n))


def test_streaming_index_golden(golden):
    g = golden("index")
    k = 0
    while f"stream_img_{k}" in g:
        img = g[f"stream_img_{k}"]
        L = int(g[f"stream_L_{k}"])
        got = O.streaming_index(O.map_from_2d(img), L)
        ref = g[f"stream_idx_{k}"]
        assert got.dtype == np.float64
        assert got.tobytes() == ref.tobytes(), k
        k += 1
    assert k == 10


def test_streaming_allocations_known():
    # n=64,L=64 -> [32,16,8,4,2,1,1]; n=32 -> [16,8,4,2,1,1]
    assert [a for a in O.streaming_allocations([4096, 1024, 256, 64, 16, 4, 1, 0, 0, 0], 64) if a] == \
        [32, 16, 8, 4, 2, 1, 1]
    assert [a for a in O.streaming_allocations([1024, 256, 64, 16, 4, 1, 0, 0, 0, 0], 32) if a] == \
        [16, 8, 4, 2, 1, 1]


def test_traditional_index_golden(golden):
    g = golden("index")
    assert [tuple(x) for x in g["trad_alloc_32"]] == O.traditional_allocation(32)
    assert [tuple(x) for x in g["trad_alloc_64"]] == O.traditional_allocation(64)
    k = 0
    while f"trad_img_{k}" in g:
        got = O.traditional_index(g[f"trad_img_{k}"], int(g[f"trad_L_{k}"]))
        ref = g[f"trad_idx_{k}"]
        assert got.dtype == ref.dtype == np.float32
        assert got.tobytes() == ref.tobytes(), k
        k += 1
    assert k == 7


def test_rag_rows_golden(golden):
    g = golden("index")
    k = 0
    while f"rag_img_{k}" in g:
        got = O.rag_multi_level_indices(g[f"rag_img_{k}"])
        ref = g[f"rag_rows_{k}"]
        assert got.dtype == ref.dtype
        assert got.tobytes() == ref.tobytes(), k
        k += 1
    assert k == 5


def test_quantize_pipeline_golden(golden):
    g = golden("quant")
    for tag in ["d1536", "d1024", "d300", "d4096"]:
        P = g[f"{tag}_params"]
        n = O.optimal_dimensions(P.shape[1])[0]
        img = O.map_to_2d(O.pad_parameters(P, n), n)
        idx = O.streaming_index(O.map_from_2d(img), n)
        assert idx.tobytes() == g[f"{tag}_idx"].tobytes()
        enh = O.embed_index_row(img, idx)
        u8, mn, mx = O.normalize_u8(enh)
        assert u8.tobytes() == g[f"{tag}_frames"].tobytes(), tag
        assert mn.tobytes() == g[f"{tag}_min"].tobytes()
        assert mx.tobytes() == g[f"{tag}_max"].tobytes()
        de = O.denormalize_u8(u8[0], mn[0], mx[0])
        assert de.tobytes() == g[f"{tag}_denorm0"].tobytes()
    u8, _, _ = O.normalize_u8(np.full((5, 4), 2.5, dtype=np.float32))
    assert u8.tobytes() == g["const_frame"].tobytes()


# ---------------------------------------------------------------- S rows


def test_parse_structure_golden(golden):
    g = golden("search")
    got = []
    for L in list(range(1, 130)) + [256, 1024, 4096]:
        for (gr, s, e, off) in O.parse_index_structure(L):
            got.append((L, gr, s, e, int(off)))
    np.testing.assert_array_equal(np.array(got), g["parse_struct"])
    assert O.segment_bounds(64) == [(0, 32), (32, 40), (40, 43), (43, 44), (44, 64)]
    assert O.segment_bounds(32) == [(0, 16), (16, 20), (20, 21), (21, 32)]


@pytest.mark.parametrize("tag", ["L64", "L32"])
def test_scores_golden(golden, tag):
    g = golden("search")
    C, Q = g[f"{tag}_C"], g[f"{tag}_Q"]
    per, ov = g[f"{tag}_per_level"], g[f"{tag}_overall"]
    for a in range(len(Q)):
        for lv in range(per.shape[2]):
            s = O.level_similarity(Q[a], C, lv)
            np.testing.assert_allclose(s, per[a, :, lv], rtol=0, atol=1e-12)
            # exact-value branches are bit-exact
            exact = np.isin(per[a, :, lv], [0.0, 0.1, 1.0])
            assert np.array_equal(s[exact], per[a, exact, lv])
        o, _ = O.overall_similarity(Q[a], C)
        np.testing.assert_allclose(o, ov[a], rtol=0, atol=1e-12)


@pytest.mark.parametrize("tag", ["L64", "L32"])
def test_search_orders_golden(golden, tag):
    g = golden("search")
    C, Q = g[f"{tag}_C"], g[f"{tag}_Q"]
    for a in range(len(Q)):
        ids, sc, _ = O.brute_force_search(Q[a], C, 10)
        np.testing.assert_array_equal(ids, g[f"{tag}_bf_ids"][a][: len(ids)])
        np.testing.assert_allclose(sc, g[f"{tag}_bf_sc"][a][: len(ids)], atol=1e-12)
        ids, sc, _, err = O.progressive_search(Q[a], C, 10, 0.1, 20)
        ref_ids = g[f"{tag}_pg_ids"][a]
        ref_ids = ref_ids[ref_ids >= 0]
        np.testing.assert_array_equal(ids, ref_ids)
        np.testing.assert_allclose(sc, g[f"{tag}_pg_sc"][a][: len(ids)], atol=1e-12)
        np.testing.assert_allclose(err, g[f"{tag}_pg_err"][a][: len(ids)], atol=1e-12)
    ids, sc, _, _ = O.progressive_search(Q[3], g[f"{tag}_fallback_C"], 10, 0.1, 20)
    np.testing.assert_array_equal(ids, g[f"{tag}_fallback_ids"])
    np.testing.assert_allclose(sc, g[f"{tag}_fallback_sc"], atol=1e-12)


@pytest.mark.parametrize("tag", ["L64", "L32", "L256"])
def test_scores_f32_golden(golden, tag):
    """float32 index vectors (and a float64 query against them): every level score, its Python type
    and the overall score bit-identical to the reference (tests/golden/search_f32.npz), including
    inexact constants, 1-ulp near-constants, f32 underflow and a large mean / std ratio."""
    g = golden("search_f32")
    C, Q = g[f"{tag}_C"], g[f"{tag}_Q"]
    assert C.dtype == np.float32
    for qtag, QQ in [("q32", Q), ("q64", Q.astype(np.float64))]:
        per, ov = g[f"{tag}_{qtag}_per_level"], g[f"{tag}_{qtag}_overall"]
        for a in range(len(QQ)):
            o, p = O.overall_similarity(QQ[a], C)
            np.testing.assert_array_equal(p, per[a], err_msg=f"{tag} {qtag} q{a}")
            np.testing.assert_array_equal(O.level_types(p, QQ.dtype == np.float32),
                                          g[f"{tag}_{qtag}_per_level_f32"][a].astype(bool))
            np.testing.assert_array_equal(o, ov[a], err_msg=f"{tag} {qtag} q{a} overall")


@pytest.mark.parametrize("tag", ["L64", "L32", "L256"])
def test_search_orders_f32_golden(golden, tag):
    g = golden("search_f32")
    C, Q = g[f"{tag}_C"], g[f"{tag}_Q"]
    for a in range(len(Q)):
        ids, sc, _ = O.brute_force_search(Q[a], C, 10)
        np.testing.assert_array_equal(ids, g[f"{tag}_pool32_bf_ids"][a][: len(ids)])
        np.testing.assert_array_equal(sc, g[f"{tag}_pool32_bf_sc"][a][: len(ids)])
        ids, sc, _, _ = O.progressive_search(Q[a], C, 10, 0.1, 20)
        ref = g[f"{tag}_pool32_pg_ids"][a]
        np.testing.assert_array_equal(ids, ref[ref >= 0])
        np.testing.assert_array_equal(sc, g[f"{tag}_pool32_pg_sc"][a][: len(ids)])


def test_f32_threshold_and_typed_overall_host_logic():
    """The threshold typing the exact kernels apply per pair (hq_search.hip typed_pass: a numpy float32
    level score against float32(threshold), a Python-float score against the threshold itself), checked
    against NumPy's own comparisons (NEP 50) around thresholds where float32(t) < t and > t; and the typed
    weighted sum of the host helper against NumPy."""
    from hq_mi355x.core.search_engine import combine_levels
    for t in (0.1, 0.3, 0.7, 0.123456789, 0.5, 1e-46, 0.95, 0.9071843218803406):
        t32 = float(np.float32(t))
        assert (t32 < t) or (t32 > t) or t32 == t
        for mode in (1, 2):
            for v in (np.nextafter(np.float32(t), np.float32(-1)), np.float32(t), np.nextafter(np.float32(t), np.float32(2))):
                want = bool(v >= t) if mode == 1 else bool(v > t)       # numpy float32 vs Python float
                got = (float(v) >= t32) if mode == 1 else (float(v) > t32)  # typed_pass, float32 score
                assert want == got, (t, mode, v)
            for p in (0.0, 0.1, 1.0, t32):                               # Python-float scores: float64
                want = (p >= t) if mode == 1 else (p > t)
                assert want == ((float(p) >= t) if mode == 1 else (float(p) > t))
    rng = np.random.default_rng(3)
    lv = rng.uniform(0, 1, (50, 5)).astype(np.float32).astype(np.float64)
    lv[:5] = 0.1
    lv[5:10, 0] = 1.0
    lv[10:15, 2] = 0.0
    got = combine_levels(lv, True)
    for i in range(len(lv)):
        tws, tw = 0.0, 0.0
        for l in range(5):
            v = lv[i, l]
            v = float(v) if v in (0.0, 0.1, 1.0) else np.float32(v)
            w = 1.0 / (l + 1)
            tws += v * w
            tw += w
        want = max(0.0, min(1.0, tws / tw))
        assert got[i] == float(want), i


def test_rag_scoring_golden(golden):
    g = golden("rag_score")
    got = O.rag_cosine(g["cos_B"], g["cos_A"])
    np.testing.assert_allclose(got, g["cos"], atol=1e-7)
    np.testing.assert_allclose(O.rag_granularity_weights(3), g["ml_w3"], atol=1e-15)
    np.testing.assert_allclose(O.rag_granularity_weights(5), g["ml_w5"], atol=1e-15)
    got = O.rag_multi_level_similarity(g["ml_Q"], g["ml_C"])
    np.testing.assert_allclose(got, g["ml"], atol=1e-12)


# ---------------------------------------------------------------- §8f row 3: pre-computed index

PRE_NAMES = ["n2", "n4", "n8", "n16", "n32", "n64", "n128", "pad1536", "const32", "f64_16"]


@pytest.mark.parametrize("name", PRE_NAMES)
def test_precomputed_index_golden(golden, name):
    g = golden("precomputed")
    img = g[f"img_{name}"]
    avg, meta = O.precomputed_index(img)
    assert avg[0].tobytes() == g[f"avg_{name}"].tobytes()
    assert [(a, b, c) for (a, b, c, _) in meta] == [tuple(r) for r in g[f"meta_{name}"]]
    n = img.shape[0]
    xy = [xy for (gg, s, _, _) in meta for xy in O.precomputed_squares(n, gg, s)]
    assert np.array_equal(np.array(xy, dtype=np.int64).reshape(-1, 2), g[f"xy_{name}"].reshape(-1, 2))
    # storage accounting (:98): averages bytes + 16 per coordinate pair
    assert int(g[f"bytes_{name}"]) == sum(4 * c + 16 * c for (_, _, c, _) in meta)
    if name in ("n16", "n64", "pad1536", "const32"):
        # the reference-shaped port bench.py times as the precomputed leg's cpu_baseline
        from oracle import hq_loops as HL
        assert HL.precomputed_one(O.map_from_2d(img), n).tobytes() == g[f"avg_{name}"].tobytes()


def test_precomputed_similarity_golden(golden):
    g = golden("precomputed")
    q, _ = O.precomputed_index(g["img_pad1536"])
    C, meta = O.precomputed_index(g["sim_cands"])
    ql = [q[0, o:o + c] for (_, _, c, o) in meta]
    for i in range(len(C)):
        cl = [C[i, o:o + c] for (_, _, c, o) in meta]
        ov, sims = O.precomputed_similarity(ql, cl)
        assert float(ov) == g["sim_overall"][i], i
        assert (0 if isinstance(ov, np.float32) else 1) == g["sim_type"][i], i
        assert [float(s) for s in sims] == list(g["sim_levels"][i]), i
    a = np.full(5, 0.5, dtype=np.float32)
    for v, want in zip(g["lvl_const_pairs"], g["lvl_const_vals"]):
        assert float(O.precomputed_level_similarity(a, np.full(5, v, dtype=np.float32))) == want


def test_reference_shaped_loops_match_oracle():
    """oracle/hq_loops.py (the per-element reference-shaped CPU port timed by bench.py's cpu_baseline) gives
    the vectorised oracle's frames and the golden's index; its candidate loop ranks like the oracle."""
    from oracle import hq_loops as HL
    rng = np.random.default_rng(8)
    for d, n in ((1536, 64), (1024, 32), (300, 32)):
        p = rng.standard_normal(d).astype(np.float32)
        img = O.map_to_2d(O.pad_parameters(p, n), n)
        u8, _, _ = O.normalize_u8(O.embed_index_row(img, O.streaming_index(O.map_from_2d(img), n)))
        assert HL.quantize_one(p, n, n).tobytes() == u8.tobytes()
        assert np.array_equal(HL.map_from_2d(HL.map_to_2d(O.pad_parameters(p, n), n)), O.pad_parameters(p, n))
    C = rng.standard_normal((300, 64))
    for a in (3, 77):
        q = C[a] + rng.normal(0, 0.01, 64)
        rid, _, _, _ = O.progressive_search(q, C, 10, 0.1, 20)
        assert HL.progressive_search(q, C, 10, 0.1, 20) == list(rid)


def test_rag_spatial_and_threshold_oracle_golden(golden):
    """Oracle restatement of the RAG scorer's height detection, spatial locality on enhanced images
    (rag/search/engine.py:134-162, 604-714) and progressive threshold (:243-287) vs the reference's goldens."""
    g = golden("rag_score")
    for tag in ("s64f", "s64d", "s32f", "s8d"):
        enh = g[f"{tag}_enh"]
        assert [O.rag_detect_height(e) for e in enh] == list(g[f"{tag}_heights"])
        for a in range(2):
            got = [O.rag_spatial_locality_enhanced(enh[a], enh[b]) for b in range(len(enh))]
            np.testing.assert_allclose(got, g[f"{tag}_spatial"][a], atol=1e-6 if enh.dtype == np.float32 else 1e-12)
    t = g["tiny_enh"]
    assert abs(O.rag_spatial_locality_enhanced(t[0], t[1]) - g["tiny_spatial"][0]) < 1e-12
    sc, ids = g["thr_scores"], g["thr_ids"]
    for level in range(5):
        for cut in (200, 37, 1):
            got = O.rag_progressive_threshold(list(zip(ids[:cut].tolist(), sc[:cut].tolist())), level)
            ref = g[f"thr_l{level}_n{cut}"]
            assert got == list(ref[ref >= 0]), (level, cut)
