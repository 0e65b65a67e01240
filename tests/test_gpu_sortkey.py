"""Python's mixed-type sort keys (tests/golden/sortkey.npz, written by the reference; make_golden.py
sortkey_fixtures): under NumPy 2 (NEP 50) the reference's sorts compare a numpy float32 score with a
Python-float score in float32 (core/search_engine.py:291 level-0 filter, :387 final sort), so a float32
score equal to float32(0.1) ties the Python 0.1 of the one-constant-side branch, and a float32 overall equal
to the float32 rounding of an all-constant-branch Python-float overall ties it; ties keep the pool order.
All-float32 searches rank by float32-rounded keys (IndexCorpus.key32, HQ_THR_KEY32,
hq_progressive_final_ex flag 1); the crafted pairs make the f64 order and Python's order differ."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TAGS = ["lv0_PF", "lv0_FP", "ov_PF", "ov_FP"]


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def _pool(C):
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    return [QuantizedModel(b"x", (8, 8), 1, 0.8, C[i], ModelMetadata(f"m{i}", 1, 1, 1.0, "t")) for i in range(len(C))]


@pytest.mark.parametrize("tag", TAGS)
def test_dropin_engine_sort_keys_golden(hq_lib, golden, tag):
    from hq_mi355x.core import ProgressiveSimilaritySearchEngine
    g = golden("sortkey")
    q, C, M = g[f"{tag}_q"], g[f"{tag}_C"], int(g[f"{tag}_M"])
    K = len(g[f"{tag}_pg_ids"])
    eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=M)
    pool = _pool(C)
    r = eng.progressive_search(q, pool, K)
    assert [int(x.model.model_id[1:]) for x in r] == list(g[f"{tag}_pg_ids"])
    np.testing.assert_array_equal([x.similarity_score for x in r], g[f"{tag}_pg_sc"])
    b = eng.brute_force_search(q, pool, K)
    assert [int(x.model.model_id[1:]) for x in b] == list(g[f"{tag}_bf_ids"])
    np.testing.assert_array_equal([x.similarity_score for x in b], g[f"{tag}_bf_sc"])
    for i in range(len(C)):
        assert eng.compare_indices_at_level(q, C[i], 0) == g[f"{tag}_lv0"][i]


@pytest.mark.parametrize("tag", ["lv0_PF", "lv0_FP"])
def test_dense_select_sort_keys_golden(hq_lib, golden, tag):
    """The dense exact path (the redo of unresolved queries) ranks level 0 by the same float32 keys: its
    top-M over the pool is the reference's level-0 survivor set and order."""
    import torch
    from hq_mi355x.core.search_engine import IndexCorpus
    g = golden("sortkey")
    q, C, M = g[f"{tag}_q"], g[f"{tag}_C"], int(g[f"{tag}_M"])
    corpus = IndexCorpus(C)
    qp = corpus.prepare_queries(q[None])
    assert corpus.key32(qp)
    s, ids, _, _ = corpus._dense(qp, torch.arange(1, device=qp.Z.device), 0, M, 0.1, 1)
    lv0 = g[f"{tag}_lv0"]
    keys = lv0.astype(np.float32)
    want = sorted([i for i in range(len(C)) if (lv0[i] >= 0.1 if lv0[i] in (0.0, 0.1, 1.0) else keys[i] >= np.float32(0.1))],
                  key=lambda i: (-keys[i], i))[:M]
    assert list(_np(ids)[0]) == want
    assert sorted(want) == sorted(g[f"{tag}_pg_ids"].tolist())  # the reference's survivors (final order: overall)


def test_sort_keys_f64_pool_unchanged(hq_lib, golden):
    """A float64 copy of the same pool compares in float64 (no numpy float32 scores): the keys stay exact."""
    from hq_mi355x.core.search_engine import IndexCorpus
    g = golden("sortkey")
    C = g["ov_PF_C"].astype(np.float64)
    q = g["ov_PF_q"].astype(np.float64)
    corpus = IndexCorpus(C)
    assert not corpus.key32(corpus.prepare_queries(q[None]))


@pytest.mark.parametrize("M", [20, 100])
@pytest.mark.parametrize("tag", ["lv0_PF", "lv0_FP"])
def test_sort_keys_scan_path_equals_dense(hq_lib, golden, tag, M):
    """The crafted float32(0.1) level-0 tie on the scan path: the golden pool padded with 150 rows that fail
    level 0 (anti-correlated copies of the query) so the scan and the lane-cooperative re-rank run (M = 20:
    the short-list kernel, M = 100: the long-list kernels); the tie row passes (`>=` in float32) and every
    output equals the dense exact path's, which test_dense_select_sort_keys_golden pins to the reference."""
    import torch
    from hq_mi355x.core.search_engine import IndexCorpus
    g = golden("sortkey")
    q, C = g[f"{tag}_q"], g[f"{tag}_C"]
    rng = np.random.default_rng(61)
    pad = (-q[None] + rng.normal(0, 0.01, (150, q.size))).astype(np.float32)
    corpus = IndexCorpus(np.concatenate([C, pad]))
    Q = np.repeat(q[None], 3, 0)
    got = [_np(x) for x in corpus.progressive(Q, 10, 0.1, M)]
    qp = corpus.prepare_queries(Q)
    assert corpus.key32(qp)
    s0, ids, best, bid = corpus._dense(qp, torch.arange(3, device=qp.Z.device), 0, M, 0.1, 1)
    oid, odet, ocnt = corpus._final(qp, s0, ids, best, bid, 10)
    want = [_np(x) for x in (oid, odet[..., 0], odet[..., 1:], ocnt)]
    for x, y in zip(got, want):
        np.testing.assert_array_equal(x, y)
    # the reference's survivors at M = 7 (the tie row among them) are all among the longer lists' results
    assert set(g[f"{tag}_pg_ids"].tolist()) <= set(got[0][0][: got[3][0]].tolist())
