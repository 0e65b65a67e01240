"""GPU parity of the level score for float32 index vectors.

The reference's compare_indices_at_level (core/search_engine.py:137-189) runs np.std / np.mean on
the arrays it is given; for f32 index vectors those are f32 reductions.  A segment that is constant
at a value whose f32 pairwise sum is inexact (64 x 0.1f: np.std = 7.45e-9, f64: 0.0) then takes the
normalised branch instead of the zero-variance one.  The checker below applies the reference's
expression to the f32 arrays with NumPy (the reference's own arithmetic) at the tolerance the
north star states (1e-5)."""
import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _ref_level(q, c):
    """core/search_engine.py:137-189 on the given arrays (f32 stays f32 inside NumPy)."""
    qs, cs = np.std(q), np.std(c)
    if qs == 0 and cs == 0:
        return 1.0 if abs(np.mean(q) - np.mean(c)) < 1e-6 else 0.0
    if qs == 0 or cs == 0:
        return 0.1
    qn = (q - np.mean(q)) / qs
    cn = (c - np.mean(c)) / cs
    sim = (np.mean(qn * cn) + 1.0) / 2.0
    mse = np.mean((q - c) ** 2)
    mx = np.mean(q ** 2) + np.mean(c ** 2)
    ds = max(0.0, 1.0 - (mse / mx)) if mx > 0 else 1.0
    return max(0.0, min(1.0, 0.7 * sim + 0.3 * ds))


def _corpus_f32(L, seed):
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((12, L)).astype(np.float32)
    C[1] = np.float32(0.1)              # constant, inexact f32 sum -> normalised branch in the ref
    C[2] = np.float32(1.7)
    C[3] = 0.0                          # constant, exact -> zero-variance branch in both
    C[4] = np.float32(0.5)              # exact constant
    C[5, : L // 2] = np.float32(0.1)
    C[6] = C[1]
    return C


@pytest.mark.parametrize("L", [64, 256])
def test_f32_constant_segments_follow_reference(L):
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x._dev import to_np
    C = _corpus_f32(L, 7)
    segs = O.parse_index_structure(L, L)
    assert segs
    corpus = IndexCorpus(C)
    for qi in (1, 2, 3, 5, 8):
        q = C[qi]
        for lvl, (_, a, b, _) in enumerate(segs):
            got = to_np(corpus.level_scores(q[None], lvl))[0]
            want = np.array([_ref_level(q[a:b], C[j, a:b]) for j in range(len(C))])
            np.testing.assert_allclose(got, want, atol=TOL, rtol=0,
                                       err_msg=f"L={L} query={qi} level={lvl}")


def test_f32_flag_changes_only_inexact_constants():
    """The same data widened to f64 keeps the f64 branches (zero variance for every constant)."""
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x._dev import to_np
    L = 256  # level 0 = 128 values: 128 x 0.1f has a non-zero f32 std
    C = _corpus_f32(L, 3)
    C64 = C.astype(np.float64)
    a, b = O.parse_index_structure(L, L)[0][1:3]
    s32 = to_np(IndexCorpus(C).level_scores(C[8][None], 0))[0]
    s64 = to_np(IndexCorpus(C64).level_scores(C64[8][None], 0))[0]
    want64 = O.level_similarity(C64[8], C64, 0)
    np.testing.assert_allclose(s64, want64, atol=1e-10, rtol=0)
    assert s64[1] == pytest.approx(0.1) and s32[1] != pytest.approx(0.1)
    for j in (0, 3, 4, 7, 9):
        assert abs(s32[j] - s64[j]) < TOL
