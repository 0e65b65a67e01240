"""Long candidate lists on the scan path (k + slack > 64): the reference engine's default
max_candidates_per_level = 100 (core/search_engine.py:31, core/video_search.py:48) and SearchConfig's 1000
(config.py:181).  The level-0 split scan fills per-query pools, k_pool_sort orders them in LDS, the tiled
exact re-rank (k_refine_big) proves the list complete, k_progressive_final_big ranks the survivors; results
are identical (ids, order, scores) to the oracle's reference-order restatement, and only queries the scan
cannot model (zero-variance queries, nothing passing) take the dense exact path."""
import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def _corpus(n_rows, L, seed):
    """Streaming-index corpus (cfg3's index shape) with degenerate rows and duplicates (ties)."""
    rng = np.random.default_rng(seed)
    d = 1536 if L == 64 else L * L
    P = rng.standard_normal((n_rows, d)).astype(np.float32)
    C = O.streaming_index(O.map_from_2d(O.map_to_2d(O.pad_parameters(P, L), L)), L)
    C[1] = 0.0
    C[2] = 0.1
    C[3] = C[17]
    C[30:34] = C[20]
    C[n_rows - 5:] = C[40]          # duplicates far apart: ties ordered by id
    return C


def _dense_counter(corpus):
    """Count the query rows the corpus sends to the dense exact path."""
    calls = []
    orig = corpus._dense

    def wrapped(qp, sel, *a, **kw):
        calls.append(int(sel.numel()))
        return orig(qp, sel, *a, **kw)

    corpus._dense = wrapped
    return calls


@pytest.mark.parametrize("kout", ["10", "full"])
@pytest.mark.parametrize("M", [100, 1000])
def test_long_list_progressive_matches_oracle(hq_lib, M, kout):
    """kout 10: the final ranking's arg-max rounds (K <= 32, tied duplicates ranked by list position);
    full: its whole-list sort."""
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(40000, 64, 21)
    rng = np.random.default_rng(22)
    Q = np.concatenate([C[[20, 3, 40, 1]] + 0.0, C[500:505] + rng.normal(0, 0.01, (5, 64)),
                        rng.standard_normal((2, 64))])
    corpus = IndexCorpus(C)
    assert M + corpus.SLACK <= corpus._max_list(0)  # the scan path, not the dense fallback
    dense = _dense_counter(corpus)
    K_out = 10 if kout == "10" else min(M, 200)
    ids, ov, lv, cnt = [_np(x) for x in corpus.progressive(Q, K_out, 0.1, M)]
    # only the zero-variance query (row 1) may need the dense exact path
    assert sum(dense) <= 1, dense
    for a in range(len(Q)):
        rid, rsc, rlv, _ = O.progressive_search(Q[a], C, K_out, 0.1, M)
        assert cnt[a] == len(rid), a
        assert list(ids[a][: cnt[a]]) == list(rid), a
        np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=TOL)
        np.testing.assert_allclose(lv[a][: cnt[a]], rlv, atol=TOL)
        assert all(ids[a][cnt[a]:] == -1)


def test_long_list_fallback_and_threshold(hq_lib):
    """Nothing passes (threshold 0.999): the first arg-max fallback; a high threshold cutting the list."""
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(20000, 64, 23)
    rng = np.random.default_rng(24)
    Q = np.concatenate([rng.standard_normal((2, 64)), C[[100, 20]] + 0.001])
    corpus = IndexCorpus(C)
    for thr in (0.999, 0.6):
        ids, ov, lv, cnt = [_np(x) for x in corpus.progressive(Q, 150, thr, 100)]
        for a in range(len(Q)):
            rid, rsc, rlv, _ = O.progressive_search(Q[a], C, 150, thr, 100)
            assert list(ids[a][: cnt[a]]) == list(rid), (thr, a)
            np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=TOL)


def test_long_list_sampled_threshold(hq_lib):
    """A corpus large enough for the 1/16 sample (stride 16): K' < k (24 at k = 108), pools sized from
    the sample; queries resolved on the scan path and equal to the oracle."""
    from hq_mi355x.core.search_engine import IndexCorpus
    rng = np.random.default_rng(25)
    N = 70000
    C = rng.standard_normal((N, 64))
    C[N - 3:] = C[77]
    Q = np.concatenate([C[[77, 1000, 5000]] + rng.normal(0, 0.02, (3, 64)), rng.standard_normal((2, 64))])
    corpus = IndexCorpus(C)
    dense = _dense_counter(corpus)
    ids, ov, lv, cnt = [_np(x) for x in corpus.progressive(Q, 100, 0.1, 100)]
    assert sum(dense) == 0, dense
    for a in range(len(Q)):
        rid, rsc, rlv, _ = O.progressive_search(Q[a], C, 100, 0.1, 100)
        assert list(ids[a][: cnt[a]]) == list(rid), a
        np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=TOL)


def test_long_list_brute_force_and_frame_scan(hq_lib):
    """k > 64 on the overall scan (brute_force_search) and the strict level-0 frame scan."""
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(30000, 64, 26)
    rng = np.random.default_rng(27)
    Q = np.concatenate([C[[20, 40]] + 0.0, C[900:903] + rng.normal(0, 0.01, (3, 64))])
    corpus = IndexCorpus(C)
    corpus.reset_stats()
    bids, bov, blv = [_np(x) for x in corpus.brute_force(Q, 120)]
    fids, fsc = [_np(x) for x in corpus.frame_search(Q, 300, 0.1)]
    # long lists stay on the scan path (the overall scan's appends go straight to the pools for k > 64)
    assert corpus.stats["dense_queries"] == 0, corpus.stats
    for a in range(len(Q)):
        rid, rsc, rlv = O.brute_force_search(Q[a], C, 120)
        assert list(bids[a]) == list(rid), a
        np.testing.assert_allclose(bov[a], rsc, atol=TOL)
        np.testing.assert_allclose(blv[a], rlv, atol=TOL)
        rid, rsc = O.hierarchical_frame_search(Q[a], C, 300, 0.1)
        assert list(fids[a][: len(rid)]) == list(rid), a
        np.testing.assert_allclose(fsc[a][: len(rid)], rsc, atol=TOL)


def test_long_list_sharded_merge_equals_single(hq_lib):
    """R = 3 shards at M = 100: records merged by hq_progressive_final (M > 64 form) == unsharded."""
    import torch
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus, shard_range
    C = _corpus(12000, 64, 28)
    C[9000:9004] = C[10]
    Q = np.concatenate([C[[10, 20, 11999]], C[[5, 6]] + 0.01])
    ref = [_np(x) for x in IndexCorpus(C).progressive(Q, 100, 0.1, 100)]
    recs = []
    for r in range(3):
        a, b = shard_range(len(C), r, 3)
        sh = ShardedIndexCorpus(C[a:b], id_base=a, n_total=len(C))
        recs.append(sh.local_records(sh.local.prepare_queries(Q), 100, 0.1))
    oid, ov, lv, cnt = ShardedIndexCorpus.merge(torch.stack(recs, 0), 100, 100)
    assert np.array_equal(_np(oid), ref[0]) and np.array_equal(_np(cnt), ref[3])
    np.testing.assert_array_equal(_np(ov), ref[1])
    np.testing.assert_array_equal(_np(lv), ref[2])


@pytest.mark.parametrize("mem", [0, 1])
@pytest.mark.parametrize("k", [65, 100, 600])
def test_pool_sort_equals_short_select_order(hq_lib, hq_option, k, mem):
    """k > 64 through k_pool_sort + the long-list re-rank: every query whose list is proven complete returns
    exactly the dense exact select's top-k (hq_level_scores + hq_select_topk: score desc, id asc), and at
    most one query is left unresolved.  mem = 1 (option pool_sort_mem): the radix select reads the pool from
    memory, the form of pools above the LDS capacity (4096 keys)."""
    hq_option("pool_sort_mem", mem)
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(25000, 64, 29)
    rng = np.random.default_rng(30)
    Q = C[300:340] + rng.normal(0, 0.01, (40, 64))
    corpus = IndexCorpus(C)
    qp = corpus.prepare_queries(Q)
    sc, ids, cnt, res = corpus._scan_refine(qp, 0, k, 0.1, 1)
    dsc, dids, _, _ = K.select_topk(K.level_scores(qp, corpus.prep, 0), k, 0.1, 1)
    res, ids, dids = _np(res), _np(ids), _np(dids)
    assert res.sum() >= len(Q) - 1
    for a in range(len(Q)):
        if res[a]:
            assert list(ids[a]) == list(dids[a]), a


@pytest.mark.parametrize("L", [64, 256])
@pytest.mark.parametrize("f32", [False, True])
def test_dense_level_scores_lds_equal_per_pair_kernel(hq_lib, hq_option, f32, L):
    """The coalesced dense scorer (k_level_scores_lds: candidate segments staged in LDS) is bit-identical
    to the one-thread-per-pair kernel (option level_scores_v1) at every level, ragged N and Q, float64
    and float32 index vectors (incl. zero-variance rows), L = 64 and 256 (a 128-value level-0 segment: 132 KB
    of staged rows, above the 64 KB default LDS allocation); and equal to the reference goldens' values via
    the oracle on a sample."""
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(3001, 64, 31) if L == 64 else np.random.default_rng(31).standard_normal((1501, L))
    if L != 64:
        C[1] = 0.0
        C[2] = 0.1
    rng = np.random.default_rng(32)
    Q = np.concatenate([C[[1, 2, 20]] + 0.0, C[100:106] + rng.normal(0, 0.01, (6, L))])
    if f32:
        C, Q = C.astype(np.float32), Q.astype(np.float32)
    corpus = IndexCorpus(C)
    for lv in range(corpus.nseg):
        got = _np(corpus.level_scores(Q, lv))
        hq_option("level_scores_v1", 1)
        want = _np(corpus.level_scores(Q, lv))
        hq_option("level_scores_v1", None)
        assert np.array_equal(got, want), lv
        for a in (0, 3, 8):
            np.testing.assert_array_equal(got[a, :500], O.level_similarity(Q[a], C[:500], lv))


@pytest.mark.parametrize("coop", [1, 0])
@pytest.mark.parametrize("kind", ["f64", "f32", "mixed"])
def test_fused_query_prepare_equals_two_launches(hq_lib, hq_option, kind, coop):
    """hq_seg_prepare_pack0 (query batches: statistics, normalised rows and split level-0 copies in one
    launch) writes exactly what hq_seg_prepare_rows + hq_seg_pack0_split write, pad rows included."""
    from hq_mi355x import kernels as K
    from hq_mi355x._dev import to_dev
    C = _corpus(1003, 64, 33)
    flags = None
    if kind == "f32":
        C = C.astype(np.float32)
    elif kind == "mixed":
        flags = np.arange(len(C)) % 3 == 0
    x = to_dev(C if kind != "mixed" else C.astype(np.float64))
    f32 = kind == "f32"
    hq_option("prep_coop", coop)  # 1: lane-cooperative statistics (default), 0: one lane per segment
    a = K.seg_prepare_pack0(x, src_f32=f32, row_f32=flags)
    b = K.pack0(K.seg_prepare(x, src_f32=f32, row_f32=flags))
    for name in ("Z", "S", "Z16", "S32"):
        assert np.array_equal(_np(getattr(a, name)).view(np.uint8), _np(getattr(b, name)).view(np.uint8)), name
    assert (a.f32, a.all32) == (b.f32, b.all32)


@pytest.mark.parametrize("rank_ct", [1, 0, 2])
@pytest.mark.parametrize("L", [32, 64, 128])
@pytest.mark.parametrize("kind", ["f64", "f32", "mixed"])
def test_cooperative_rerank_equals_per_thread_kernel(hq_lib, hq_option, L, kind, rank_ct):
    """The lane-cooperative long-list re-rank (k_refine_coop: 8 lanes per entry, NumPy's eight pairwise
    accumulators one per lane, rows staged per group) is bit-identical to the one-thread-per-entry kernel
    (option refine_coop = 0): progressive M = 100 / 1000 (level-0 ranking + [overall, level..] records),
    brute force k > 64 (overall ranking), frame scan (strict level-0); float64, float32 and mixed pools.
    rank_ct 1 (default): the scorers specialised to the compile-time level structures of L = 64 / 32 (L = 128
    keeps the runtime form); 0: the runtime-structure scorer everywhere; 2: also in the short-list kernel."""
    from hq_mi355x.core.search_engine import IndexCorpus
    hq_option("rank_ct", rank_ct)
    C = _corpus(3000 if L == 128 else 20000, L, 41 + L)
    rng = np.random.default_rng(42)
    Q = np.concatenate([C[[1, 2, 20, 40]] + 0.0, C[100:108] + rng.normal(0, 0.01, (8, L)),
                        rng.standard_normal((2, L))])
    if kind == "f32":
        C, Q = C.astype(np.float32), Q.astype(np.float32)
    corpus = IndexCorpus(C, row_f32=(np.arange(len(C)) % 3 == 0) if kind == "mixed" else None)

    def run():
        out = [_np(x) for x in corpus.progressive(Q, 150, 0.1, 100)]
        out += [_np(x) for x in corpus.progressive(Q, 1000, 0.1, 1000)]
        out += [_np(x) for x in corpus.brute_force(Q, 120)]
        out += [_np(x) for x in corpus.frame_search(Q, 300, 0.1)]
        return out

    got = run()
    hq_option("refine_coop", 0)
    want = run()
    hq_option("refine_coop", None)
    for a, (x, y) in enumerate(zip(got, want)):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (kind, L, a)


@pytest.mark.parametrize("lists", [False, True])
@pytest.mark.parametrize("kind", ["f64", "f32", "mixed"])
@pytest.mark.parametrize("L", [32, 64, 128])
def test_fused_final_ranking_equals_two_steps(hq_lib, L, kind, lists):
    """Long lists: the final ranking fused into the re-rank's sort (hq_refine_final_ws) equals the two-step
    form (hq_refine_topk_ws records + hq_progressive_final_ex) bit for bit — M = 100 and 1000, K = 10
    (arg-max rounds), 40 and 150 (sort), ties (duplicate rows), float64 / float32 / mixed pools; with and without
    the (unreturned) level-0 lists written (hq_refine_final_ws accepts NULL for them)."""
    from hq_mi355x import kernels as K_
    from hq_mi355x.core import search_engine as SE
    K_.FINAL_LEVEL0_LISTS = lists
    C = _corpus(3000 if L == 128 else 20000, L, 71 + L)
    rng = np.random.default_rng(72)
    Q = np.concatenate([C[[1, 2, 20, 40, 30]] + 0.0, C[100:108] + rng.normal(0, 0.01, (8, L)),
                        rng.standard_normal((2, L))])
    if kind == "f32":
        C, Q = C.astype(np.float32), Q.astype(np.float32)
    corpus = SE.IndexCorpus(C, row_f32=(np.arange(len(C)) % 3 == 0) if kind == "mixed" else None)

    def run():
        out = []
        for M, K_out in ((100, 10), (100, 40), (1000, 10), (1000, 150)):
            out += [_np(x) for x in corpus.progressive(Q, K_out, 0.1, M)]
        return out

    try:
        got = run()
    finally:
        K_.FINAL_LEVEL0_LISTS = True
    SE._FUSED_FINAL = False
    try:
        want = run()
    finally:
        SE._FUSED_FINAL = True
    for a, (x, y) in enumerate(zip(got, want)):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (kind, L, a)


@pytest.mark.parametrize("rank_ct", [1, 2])
@pytest.mark.parametrize("kind", ["f64", "f32", "mixed"])
@pytest.mark.parametrize("L", [32, 64, 128])
def test_short_list_rerank_equals_per_thread_kernel(hq_lib, hq_option, L, kind, rank_ct):
    """The fused short-list re-rank (k_rank_small: k_rank_pairs' lane groups and the ranking in one
    workgroup per query, lists of <= 64 entries) is bit-identical to k_refine_lds (option refine_small = 0):
    progressive M = 20 (28 entries: 32 groups) and M = 50 (58: 64 groups) with records, brute force top-10
    (overall ranking), frame scan (strict level-0); float64, float32 and mixed pools, ties included.
    rank_ct 2: k_rank_small with the compile-time level structures of L = 64 / 32."""
    from hq_mi355x.core.search_engine import IndexCorpus
    hq_option("rank_ct", rank_ct)
    C = _corpus(3000 if L == 128 else 20000, L, 51 + L)
    rng = np.random.default_rng(52)
    Q = np.concatenate([C[[1, 2, 20, 40]] + 0.0, C[100:108] + rng.normal(0, 0.01, (8, L)),
                        rng.standard_normal((2, L))])
    if kind == "f32":
        C, Q = C.astype(np.float32), Q.astype(np.float32)
    corpus = IndexCorpus(C, row_f32=(np.arange(len(C)) % 3 == 0) if kind == "mixed" else None)

    def run():
        out = [_np(x) for x in corpus.progressive(Q, 10, 0.1, 20)]
        out += [_np(x) for x in corpus.progressive(Q, 40, 0.1, 50)]
        out += [_np(x) for x in corpus.brute_force(Q, 10)]
        out += [_np(x) for x in corpus.frame_search(Q, 30, 0.1)]
        return out

    got = run()
    hq_option("refine_small", 0)
    want = run()
    hq_option("refine_small", None)
    for a, (x, y) in enumerate(zip(got, want)):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (kind, L, a)


@pytest.mark.parametrize("k", [65, 300, 1000])
def test_sort_select_equals_reference_order(hq_lib, hq_option, k):
    """The sort-based dense select for long lists (k_select_sort: LDS bitonic parts + merge stages) returns
    exactly the (score desc, id asc) top-k among entries passing the threshold test, and the first arg-max,
    for heavy ties, every threshold mode and ragged parts; identical to the k-pass two-stage select (option
    select_2stage), which it replaces for k > 64 (the dense exact path's select)."""
    import torch
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(50 + k)
    N = 70001
    sc = np.round(rng.random((3, N)), 3)  # ~1000 distinct values: long runs of ties
    sc[1, :] = 0.1                         # one row of equal scores (a zero-variance query)
    sc[2, 5000:5100] = 0.9995
    dsc = torch.from_numpy(sc).cuda()
    for thr, mode in ((0.0, 0), (0.5, 1), (0.1, 2), (0.999, 1)):
        got = [_np(x) for x in K.select_topk(dsc, k, thr, mode, 7)]
        hq_option("select_2stage", 1)
        want = [_np(x) for x in K.select_topk(dsc, k, thr, mode, 7)]
        hq_option("select_2stage", None)
        for a, b in zip(got, want):
            assert np.array_equal(a, b), (k, thr, mode)
        for r in range(3):
            ok = np.ones(N, bool) if mode == 0 else (sc[r] >= thr if mode == 1 else sc[r] > thr)
            idx = np.nonzero(ok)[0]
            order = idx[np.lexsort((idx, -sc[r][idx]))][:k]
            n = len(order)
            assert list(got[1][r][:n]) == list(order + 7) and np.all(got[1][r][n:] == -1), (k, thr, mode, r)
            assert np.array_equal(got[0][r][:n], sc[r][order])
            assert got[3][r] == int(np.argmax(sc[r])) + 7 and got[2][r] == sc[r].max()


@pytest.mark.parametrize("nt", [512, 256, "no-small"])
@pytest.mark.parametrize("dups", [0, 40])
@pytest.mark.parametrize("kind", ["f64", "f32"])
def test_window_ranking_equals_sort(hq_lib, hq_option, kind, dups, nt):
    """k_rank_sort's window ranking (option rank_win 1: each entry ranked from the approximate-score order of
    the list plus exact comparisons inside its 2-eps window, the result checked and the bitonic sort run when
    the check fails) is bit-identical to the sort alone (rank_win 0) and to the one-thread-per-entry kernels
    (refine_coop 0): progressive M = 100 / 1000 with K = 10 and 150, brute force k > 64, frame scan.
    dups 40: runs of 40 identical rows (windows past the 32-entry cap: the sort fallback on every list
    holding a run) beside distinct rows.  nt: workgroup size of the lists > 512 (option rank_sort_nt: two or four
    entries per thread; lists <= 128 take a 128-entry workgroup unless option rank_sort_small is 0)."""
    from hq_mi355x.core.search_engine import IndexCorpus
    if nt == "no-small":
        hq_option("rank_sort_small", 0)
    else:
        hq_option("rank_sort_nt", nt)
    C = _corpus(20000, 64, 91)
    if dups:
        C[1000:1000 + 50 * dups] = np.repeat(C[1000:1050], dups, axis=0)
    rng = np.random.default_rng(92)
    Q = np.concatenate([C[[1, 2, 20, 40, 30, 1000, 1000 + 3 * dups]] + 0.0,
                        C[100:106] + rng.normal(0, 0.01, (6, 64)), rng.standard_normal((2, 64))])
    if kind == "f32":
        C, Q = C.astype(np.float32), Q.astype(np.float32)
    corpus = IndexCorpus(C)

    def run():
        out = []
        for M, K_out in ((100, 10), (100, 150), (1000, 10), (1000, 150)):
            out += [_np(x) for x in corpus.progressive(Q, K_out, 0.1, M)]
        out += [_np(x) for x in corpus.brute_force(Q, 120)]
        out += [_np(x) for x in corpus.frame_search(Q, 300, 0.1)]
        return out

    got = run()
    hq_option("rank_win", 0)
    want = run()
    hq_option("refine_coop", 0)
    ref = run()
    for a, (x, y, z) in enumerate(zip(got, want, ref)):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (kind, dups, a)
        assert np.array_equal(x.view(np.uint8), z.view(np.uint8)), (kind, dups, a)
