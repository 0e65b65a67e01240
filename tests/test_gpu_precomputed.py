"""GPU parity of the pre-computed overlapping-square index (SURVEY.md §8f row 3,
core/precomputed_hilbert_index.py) against the reference's golden vectors and the oracle."""
import contextlib
import io

import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu

NAMES = ["n2", "n4", "n8", "n16", "n32", "n64", "n128", "pad1536", "const32", "f64_16"]


def _np(t):
    return t.detach().cpu().numpy()


def _t(a):
    from hq_mi355x._dev import to_dev
    return to_dev(a)


@pytest.mark.parametrize("name", NAMES)
def test_precomputed_index_golden(hq_lib, golden, name):
    from hq_mi355x import kernels as K
    g = golden("precomputed")
    img = g[f"img_{name}"]
    n = img.shape[0]
    avg = K.precomputed_index(_t(img[None]), n, 0)
    assert _np(avg)[0].tobytes() == g[f"avg_{name}"].tobytes()
    lay = K.precomputed_layout(n)
    assert [(a, b, c) for (a, b, c, _) in lay] == [tuple(r) for r in g[f"meta_{name}"]]


def test_precomputed_from_parameter_stream(hq_lib, golden):
    """kind 1: the 1-D parameters are padded and Hilbert-mapped in the kernel (_get_2d_representation)."""
    from hq_mi355x import kernels as K
    g = golden("precomputed")
    p = O.map_from_2d(g["img_pad1536"][None])[0][:1536]
    avg = K.precomputed_index(_t(np.stack([p, p * 2])), 64, 1)
    assert _np(avg)[0].tobytes() == g["avg_pad1536"].tobytes()
    want, _ = O.precomputed_index(O.map_to_2d(O.pad_parameters(np.stack([p * 2]), 64), 64))
    assert _np(avg)[1].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("n,N", [(16, 33), (32, 17), (64, 9), (128, 3)])
def test_precomputed_batch_vs_oracle(hq_lib, n, N):
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(n + N)
    imgs = (rng.standard_normal((N, n, n)) * 10 ** rng.uniform(-2, 2)).astype(np.float32)
    imgs[1] = 0.75
    want, _ = O.precomputed_index(imgs)
    assert _np(K.precomputed_index(_t(imgs), n, 0)).tobytes() == want.tobytes()


@pytest.mark.parametrize("max_levels,min_sq", [(3, 2), (6, 4), (2, 1)])
def test_precomputed_custom_levels(hq_lib, max_levels, min_sq):
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(max_levels)
    imgs = rng.standard_normal((4, 32, 32)).astype(np.float32)
    want, meta = O.precomputed_index(imgs, max_levels, min_sq)
    got = K.precomputed_index(_t(imgs), 32, 0, None, max_levels, min_sq)
    assert _np(got).tobytes() == want.tobytes()
    assert [(a, b, c, o) for (a, b, c, o) in K.precomputed_layout(32, max_levels, min_sq)] == meta


def test_precomputed_similarity_golden(hq_lib, golden):
    from hq_mi355x.core.precomputed_hilbert_index import PrecomputedHilbertIndexer, PrecomputedSimilaritySearchEngine
    g = golden("precomputed")
    ix = PrecomputedHilbertIndexer()
    eng = PrecomputedSimilaritySearchEngine(ix)
    with contextlib.redirect_stdout(io.StringIO()):
        qi = ix.create_precomputed_index(g["img_pad1536"], "q")
        cis = [ix.create_precomputed_index(c, f"c{i}") for i, c in enumerate(g["sim_cands"])]
    for i, ci in enumerate(cis):
        v = eng._calculate_precomputed_similarity(qi, ci)
        assert float(v) == g["sim_overall"][i], i
        assert (0 if isinstance(v, np.float32) else 1) == g["sim_type"][i], i
        lv = [float(eng._compare_precomputed_levels(a, b)) for a, b in zip(qi.levels, ci.levels)]
        assert lv == list(g["sim_levels"][i]), i
    from hq_mi355x.core.precomputed_hilbert_index import PrecomputedLevel
    a = PrecomputedLevel(2, 2, 5, np.full(5, 0.5, dtype=np.float32), [])
    for v, want in zip(g["lvl_const_pairs"], g["lvl_const_vals"]):
        b = PrecomputedLevel(2, 2, 5, np.full(5, v, dtype=np.float32), [])
        assert float(eng._compare_precomputed_levels(a, b)) == want


def test_precomputed_similarity_matrix_vs_oracle(hq_lib):
    """Batched Q x N similarity (one device call) == the reference arithmetic pair by pair."""
    from hq_mi355x.core.precomputed_hilbert_index import PrecomputedSimilaritySearchEngine
    rng = np.random.default_rng(4)
    base = rng.standard_normal((3, 32, 32)).astype(np.float32)
    cands = np.concatenate([base + rng.normal(0, s, base.shape).astype(np.float32) for s in (0.01, 0.3, 2.0)])
    cands[2] = 1.5  # constant image
    qa, meta = O.precomputed_index(base)
    ca, _ = O.precomputed_index(cands)
    offs = [o for (_, _, _, o) in meta]
    cnts = [c for (_, _, c, _) in meta]
    eng = PrecomputedSimilaritySearchEngine(None)
    ov, ty, lv = eng.similarity_matrix(qa, ca, offs, offs, cnts, levels=True)
    ov, ty = _np(ov), _np(ty)
    for q in range(len(qa)):
        ql = [qa[q, o:o + c] for (_, _, c, o) in meta]
        for c in range(len(ca)):
            want, _ = O.precomputed_similarity(ql, [ca[c, o:o + k] for (_, _, k, o) in meta])
            assert ov[q, c] == float(want) and ty[q, c] == (0 if isinstance(want, np.float32) else 1), (q, c)


def test_precomputed_dropin_surface(hq_lib, tmp_path):
    from hq_mi355x.core.precomputed_hilbert_index import PrecomputedHilbertIndexer, PrecomputedSimilaritySearchEngine
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    rng = np.random.default_rng(9)
    img = rng.standard_normal((64, 64)).astype(np.float32)
    ix = PrecomputedHilbertIndexer()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        idx = ix.create_precomputed_index(img, "m")
    assert "Pre-computing 6 granularity levels for m..." in buf.getvalue()
    assert ix.get_index("m") is idx and idx.total_storage_bytes == 2610 * 20
    with pytest.raises(ValueError, match="Image must be square, got 4x8"):
        ix.create_precomputed_index(np.zeros((4, 8), dtype=np.float32), "bad")
    f = tmp_path / "idx.npz"
    ix.save_index_to_disk(idx, str(f))
    back = PrecomputedHilbertIndexer().load_index_from_disk(str(f))
    assert all(a.averages.tobytes() == b.averages.tobytes() for a, b in zip(idx.levels, back.levels))
    assert abs(ix.get_storage_overhead(64 * 64 * 4) - 2610 * 12 / (64 * 64 * 4) * 100) < 1e-12
    # search(): like the reference, SearchResult(..., level_similarities={}) is rejected by the dataclass
    eng = PrecomputedSimilaritySearchEngine(ix)
    md = ModelMetadata("m", 1, 1, 1.0, "t")
    qm = QuantizedModel(b"x", (64, 64), 4096, 0.8, np.zeros(64), md)
    q = O.map_from_2d(img[None])[0]
    with contextlib.redirect_stdout(io.StringIO()):
        with pytest.raises(TypeError):
            eng.search(q, [qm])
    # a candidate without a cached index is skipped (warning), nothing passes -> []
    md2 = ModelMetadata("missing", 1, 1, 1.0, "t")
    with contextlib.redirect_stdout(io.StringIO()):
        assert eng.search(q, [QuantizedModel(b"x", (64, 64), 4096, 0.8, np.zeros(64), md2)]) == []
    # legacy comparison (np.corrcoef) within 1e-12
    a, b = rng.standard_normal(64), rng.standard_normal(64)
    assert abs(eng.compare_indices_at_level(a, b, 0) - (np.corrcoef(a, b)[0, 1] + 1) / 2) < 1e-12
    assert eng.compare_indices_at_level(np.full(8, 2.0), np.full(8, 2.0), 0) == 1.0
    assert eng.compare_indices_at_level(np.full(8, 2.0), a[:8], 0) == 0.1


def test_quantizer_builds_precomputed_index(hq_lib):
    from hq_mi355x.api import HilbertQuantizer
    pytest.importorskip("PIL")
    hq = HilbertQuantizer()
    p = np.random.default_rng(1).standard_normal(1024).astype(np.float32)
    with contextlib.redirect_stdout(io.StringIO()):
        qm = hq.quantize(p, model_id="pm")
    pre = hq.precomputed_indexer.get_index("pm")
    want, _ = O.precomputed_index(O.map_to_2d(p[None], 32))
    assert np.concatenate([lv.averages for lv in pre.levels]).tobytes() == want[0].tobytes()
    assert HilbertQuantizer(use_precomputed_indexing=False).quantize(p, model_id="x") is not None
    assert qm.metadata.model_name == "pm"


@pytest.mark.parametrize("ws", [None, 0, 3, "order0", "g2reg", "compact"])
@pytest.mark.parametrize("grid", [None, "3"])
@pytest.mark.parametrize("n,dtype,levels", [(16, np.float32, (6, 2)), (32, np.float32, (6, 2)),
                                             (64, np.float32, (6, 2)), (64, np.float64, (6, 2)),
                                             (32, np.float32, (2, 1)), (64, np.float32, (3, 4))])
def test_precomputed_stream_zero_padding_skip(hq_lib, hq_option, ws, grid, n, dtype, levels):
    """1-D streams shorter than n*n: squares wholly in the zero padding are skipped (pre_zero_plan) and
    their averages stay +0.0.  d sweeps group edges (d % 4 != 0), block edges and the full image; with
    HQ_PRECOMP_GRID=3 each workgroup loops over several images, so the padding cells and the skipped
    averages are reused from the once-per-workgroup setup.  f32 skip runs take the wave-specialised
    k_precomp_ws (loader / storer waves; 2, 3 or 4 groups per loader lane by d) unless precomp_ws = 0;
    the host-built square lists are in LDS bank order unless precomp_order = 0; its 2 x 2 grid squares are
    averaged from the LDS image unless precomp_g2reg = 1 (the loader's registers); only the listed squares'
    averages are kept in LDS (compact, mapped back to the output row by the storer waves) with
    precomp_compact = 1."""
    from hq_mi355x import kernels as K
    if grid is not None:
        hq_option("precomp_grid", int(grid))
    if ws == "order0":
        hq_option("precomp_order", 0)
    elif ws == "g2reg":
        hq_option("precomp_g2reg", 1)
    elif ws == "compact":
        hq_option("precomp_compact", 1)
    elif ws is not None:
        hq_option("precomp_ws", ws)
    rng = np.random.default_rng(n * 7 + len(levels))
    ml, ms = levels
    ds = {1, 3, 4, 5, 63, 64, 65, n * n // 4 + 1, 3 * n * n // 8, n * n - 1, n * n}
    if n == 64:
        ds |= {1023, 1024, 1537, 2047, 2048, 2049, 2050}
    for d in sorted(ds):
        p = (rng.standard_normal((7, d)) * 10 ** rng.uniform(-2, 2)).astype(dtype)
        p[2] = 0.5
        p[3, ::2] = -0.0
        want, _ = O.precomputed_index(O.map_to_2d(O.pad_parameters(p, n), n), ml, ms)
        got = _np(K.precomputed_index(_t(p), n, 1, None, ml, ms))
        assert got.tobytes() == want.tobytes(), f"n={n} d={d}"
