"""GPU parity of the similarity scan (S2-S7): scores within 1e-10 of the reference (exact for the
constant branches), rankings identical (ids and order) to the reference's stable sorts."""
import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-10  # north star: scores within 1e-5 of the reference NumPy path; we hold 1e-10


def _t(x):
    from hq_mi355x._dev import to_dev
    return to_dev(x)


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def _corpus(n_rows, L, seed, dup=True):
    """Realistic streaming-index corpus + degenerate rows (zeros, constants, duplicates)."""
    rng = np.random.default_rng(seed)
    n = L
    d = 1536 if n == 64 else n * n
    P = rng.standard_normal((n_rows, d)).astype(np.float32)
    img = O.map_to_2d(O.pad_parameters(P, n), n)
    C = O.streaming_index(O.map_from_2d(img), L)
    if dup and n_rows > 40:
        C[1] = 0.0
        C[2] = 0.1
        C[3] = C[17]
        C[4] = -C[18]
        C[5, : L // 2] = 0.25
        C[30:34] = C[20]
    return C


def test_prepare_stats_exact(hq_lib, golden):
    from hq_mi355x import kernels as K
    g = golden("search")
    for tag, L in [("L64", 64), ("L32", 32)]:
        C = g[f"{tag}_C"]
        prep = K.seg_prepare(_t(C))
        S = _np(prep.S)
        for s, (a, b) in enumerate(O.segment_bounds(L)):
            seg = C[:, a:b]
            np.testing.assert_array_equal(S[:, s, 0], O.np_mean_rows(seg))
            np.testing.assert_array_equal(S[:, s, 1], O.np_std_rows(seg))


@pytest.mark.parametrize("tag", ["L64", "L32"])
def test_level_and_overall_scores_golden(hq_lib, golden, tag):
    from hq_mi355x.core.search_engine import IndexCorpus
    g = golden("search")
    C, Q, per, ov = g[f"{tag}_C"], g[f"{tag}_Q"], g[f"{tag}_per_level"], g[f"{tag}_overall"]
    corpus = IndexCorpus(C)
    for lv in range(per.shape[2]):
        got = _np(corpus.level_scores(Q, lv))
        assert np.array_equal(got, per[:, :, lv])          # exact scores are bit-identical
    assert np.array_equal(_np(corpus.level_scores(Q, -1)), ov)


@pytest.mark.parametrize("tag", ["L64", "L32"])
def test_dropin_engine_golden(hq_lib, golden, tag):
    from hq_mi355x.core import ProgressiveSimilaritySearchEngine
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    g = golden("search")
    C, Q = g[f"{tag}_C"], g[f"{tag}_Q"]
    n = C.shape[1]

    def pool_of(M):
        return [QuantizedModel(b"x", (n, n), 1, 0.8, M[i], ModelMetadata(f"m{i}", 1, 1, 1.0, "t")) for i in range(len(M))]

    pool = pool_of(C)
    eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=20)
    for a in range(len(Q)):
        r = eng.brute_force_search(Q[a], pool, 10)
        assert [int(x.model.model_id[1:]) for x in r] == [i for i in g[f"{tag}_bf_ids"][a] if i >= 0]
        np.testing.assert_allclose([x.similarity_score for x in r], g[f"{tag}_bf_sc"][a][: len(r)], atol=TOL)
        r = eng.progressive_search(Q[a], pool, 10)
        assert [int(x.model.model_id[1:]) for x in r] == [i for i in g[f"{tag}_pg_ids"][a] if i >= 0]
        np.testing.assert_allclose([x.similarity_score for x in r], g[f"{tag}_pg_sc"][a][: len(r)], atol=TOL)
        np.testing.assert_allclose([x.reconstruction_error for x in r], g[f"{tag}_pg_err"][a][: len(r)], atol=TOL)
        assert abs(eng.compare_indices_at_level(Q[a], C[7], 0) - g[f"{tag}_per_level"][a, 7, 0]) <= TOL
    r = eng.progressive_search(Q[3], pool_of(g[f"{tag}_fallback_C"]), 10)
    assert [int(x.model.model_id[1:]) for x in r] == list(g[f"{tag}_fallback_ids"])


def test_mixed_length_pool(hq_lib):
    from hq_mi355x.core import ProgressiveSimilaritySearchEngine
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    rng = np.random.default_rng(3)
    C64 = _corpus(30, 64, 1, dup=False)
    C32 = _corpus(30, 32, 2, dup=False)
    pool = [QuantizedModel(b"x", (8, 8), 1, 0.8, v, ModelMetadata(f"m{i}", 1, 1, 1.0, "t"))
            for i, v in enumerate(list(C64) + list(C32))]
    q = C64[4] + rng.normal(0, 0.01, 64)
    eng = ProgressiveSimilaritySearchEngine(0.1, 20)
    for lv in range(5):
        for c in [C64[0], C32[0]]:
            assert abs(eng.compare_indices_at_level(q, c, lv) - O.level_similarity(q, c[None], lv)[0]) <= TOL
    r = eng.progressive_search(q, pool, 10)
    assert r[0].model.model_id == "m4"


@pytest.mark.parametrize("L", [64, 32])
def test_batched_search_vs_oracle(hq_lib, L):
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(3000, L, 7)
    rng = np.random.default_rng(9)
    Q = np.concatenate([C[[10, 20, 3, 1, 2, 5]] + 0.0, C[100:160] + rng.normal(0, 0.01, (60, L)),
                        rng.standard_normal((4, L))])
    corpus = IndexCorpus(C)
    ids, ov, lv, cnt = corpus.progressive(Q, 10, 0.1, 20)
    ids, ov, lv, cnt = _np(ids), _np(ov), _np(lv), _np(cnt)
    bids, bov, blv = [_np(x) for x in corpus.brute_force(Q, 10)]
    fids, fsc = [_np(x) for x in corpus.frame_search(Q, 10, 0.1)]
    for a in range(len(Q)):
        rid, rsc, rlv, _ = O.progressive_search(Q[a], C, 10, 0.1, 20)
        assert list(ids[a][: cnt[a]]) == list(rid)
        np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=TOL)
        np.testing.assert_allclose(lv[a][: cnt[a]], rlv, atol=TOL)
        rid, rsc, _ = O.brute_force_search(Q[a], C, 10)
        assert list(bids[a]) == list(rid)
        np.testing.assert_allclose(bov[a], rsc, atol=TOL)
        rid, rsc = O.hierarchical_frame_search(Q[a], C, 10, 0.1)
        assert list(fids[a][: len(rid)]) == list(rid) and all(fids[a][len(rid):] == -1)
        np.testing.assert_allclose(fsc[a][: len(rid)], rsc, atol=TOL)


def test_large_k_select_path(hq_lib):
    """max_candidates_per_level = 100 (the reference engine default) takes the dense + select path."""
    from hq_mi355x.core.search_engine import IndexCorpus
    C = _corpus(1500, 64, 12)
    Q = C[[7, 8, 9]] + 0.001
    ids, ov, lv, cnt = [_np(x) for x in IndexCorpus(C).progressive(Q, 10, 0.1, 100)]
    for a in range(len(Q)):
        rid, rsc, _, _ = O.progressive_search(Q[a], C, 10, 0.1, 100)
        assert list(ids[a][: cnt[a]]) == list(rid)
        np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=TOL)


def test_sharded_merge_equals_single(hq_lib):
    """R corpus shards merged by hq_progressive_final == the unsharded scan (same ids, same order)."""
    import torch
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import pack, shard_range, unpack
    C = _corpus(5000, 64, 31)
    C[4000:4010] = C[50]          # duplicates straddling shards: tie order must follow global ids
    Q = C[[50, 60, 70, 1, 2]] + 0.0
    full = IndexCorpus(C)
    ref = [_np(x) for x in full.progressive(Q, 10, 0.1, 20)]
    R = 4
    recs = []
    for r in range(R):
        a, b = shard_range(len(C), r, R)
        sh = IndexCorpus(C[a:b], id_base=a)
        qp = sh.prepare_queries(Q)
        s0, ids, _, best, bid = sh.exact_topk(qp, 0, 20, 0.1, 1, need_best=True)
        det = K.rescore(qp, sh.prep, ids, a)
        bdet = K.rescore(qp, sh.prep, bid.view(-1, 1), a)
        recs.append(torch.cat([pack(s0, ids, det), pack(best.view(-1, 1), bid.view(-1, 1), bdet)], dim=1))
    g = torch.stack(recs, 0)
    gs, gi, gd = unpack(g[:, :, :20])
    bs, bi, bd = unpack(g[:, :, 20])
    oid, odet, cnt = K.progressive_final(gs, gi, gd, bs, bi, bd, 10)
    assert np.array_equal(_np(oid), ref[0]) and np.array_equal(_np(cnt), ref[3])
    np.testing.assert_array_equal(_np(odet)[..., 0], ref[1])


def test_sharded_corpus_records_equal_single(hq_lib):
    """ShardedIndexCorpus.local_records (sync-late path, dense fix-ups) of 3 shards merged == unsharded;
    a shard where nothing passes contributes its exact arg-max slot; world size 1 without a process
    group gathers its own records."""
    import torch
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus, shard_range
    C = _corpus(3000, 64, 41)
    C[2500:2504] = C[10]
    Q = np.concatenate([C[[10, 20, 2999]], C[[5, 6]] + 0.01])
    full = IndexCorpus(C)
    for thr in (0.1, 0.97):
        ref = [_np(x) for x in full.progressive(Q, 10, thr, 20)]
        recs = []
        for r in range(3):
            a, b = shard_range(len(C), r, 3)
            sh = ShardedIndexCorpus(C[a:b], id_base=a, n_total=len(C))
            recs.append(sh.local_records(sh.local.prepare_queries(Q), 20, thr))
        oid, ov, lv, cnt = ShardedIndexCorpus.merge(torch.stack(recs, 0), 20, 10)
        assert np.array_equal(_np(oid), ref[0]) and np.array_equal(_np(cnt), ref[3]), thr
        np.testing.assert_array_equal(_np(ov), ref[1])
        one = ShardedIndexCorpus(C, id_base=0, n_total=len(C)).progressive(Q, 10, thr, 20)
        assert np.array_equal(_np(one[0]), ref[0])


def test_pipelined_submit_finish_equals_sequential(hq_lib):
    """Batches queued before the previous one is finished (progressive_submit / _finish, as bench.py
    runs them): every batch's results equal its own synchronous call, including batches whose queries
    take the dense path (nothing passes at 0.97: count-0 rows are redone after the next batch was
    queued, so the shared redo counter and scan workspace must not leak between batches)."""
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus
    C = _corpus(4000, 64, 51)
    rng = np.random.default_rng(52)
    batches = [(C[[1, 2, 3]] + rng.normal(0, 0.01, (3, 64)), 0.1), (C[[7, 8]] + 0.02, 0.97),
               (C[100:140] + rng.normal(0, 0.01, (40, 64)), 0.1), (rng.standard_normal((5, 64)), 0.97)]
    import torch
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    for corpus in (IndexCorpus(C), ShardedIndexCorpus(C, id_base=0, n_total=len(C))):
        ref = [[_np(x) for x in corpus.progressive(q, 10, thr, 20)] for q, thr in batches]
        for nst in (1, 2):  # one stream, or batches alternating between two (as bench.py runs them)
            pend, got = [], []
            for i, (q, thr) in enumerate(batches):
                st = streams[i % nst]
                with torch.cuda.stream(st):
                    pend.append((st, corpus.progressive_submit(q, 10, thr, 20)))
                if len(pend) > 1:
                    st0, p = pend.pop(0)
                    with torch.cuda.stream(st0):
                        got.append([_np(x) for x in corpus.progressive_finish(p)])
            for st0, p in pend:
                with torch.cuda.stream(st0):
                    got.append([_np(x) for x in corpus.progressive_finish(p)])
                    again = [_np(x) for x in corpus.progressive_finish(p)]  # a handle finishes once
                    assert all(np.array_equal(x, y) for x, y in zip(got[-1], again))
            torch.cuda.synchronize()
            for b, (r, g) in enumerate(zip(ref, got)):
                for x, y in zip(r, g):
                    assert np.array_equal(x, y), (type(corpus).__name__, nst, b)


def test_rag_scores(hq_lib, golden):
    from hq_mi355x.rag import similarity as S
    g = golden("rag_score")
    got = [S.calculate_embedding_cosine_similarity(g["cos_B"], g["cos_A"][i]) for i in range(8)]
    np.testing.assert_allclose(got, g["cos"], atol=1e-6)
    got = [S.compare_multi_level_indices(g["ml_Q"], g["ml_C"][i]) for i in range(6)]
    np.testing.assert_allclose(got, g["ml"], atol=1e-6)
    np.testing.assert_allclose(S.calculate_granularity_weights(5), g["ml_w5"], atol=1e-15)
    a = g["cos_A"][0]
    b = g["cos_B"]
    assert abs(S.calculate_spatial_locality_similarity(a, b) - O.rag_spatial_locality_similarity(a, b)) < 1e-6


def test_level0_scan_kernels_agree_and_match_oracle(hq_lib, hq_option):
    """The level-0 scan variants (k_scan0g at 1 or 4 waves per block, 64 or 128 queries per wave, 4 or 3 waves per SIMD and prefetch distance 2-8, the
    G-selected or full-filter sample pass or none, the list-based k_scan0f) give the same exact top-k as
    the LDS-tiled k_scan (option scan_v1) and as the oracle, on a corpus with a ragged chunk tail, zero-variance level-0 segments on both sides,
    duplicate runs across chunks and a query count that is not a multiple of 64."""
    from hq_mi355x.core.search_engine import IndexCorpus
    rng = np.random.default_rng(77)
    N, L = 40_003, 64
    C = rng.standard_normal((N, L))
    C[100:140, :32] = 0.5                      # constant level-0 segments (std 0)
    C[200:210, :32] = 0.5 + 1e-7               # |mean diff| < 1e-6 -> score 1 vs a constant query
    C[39_990:] = C[7]                          # duplicates in the last (ragged) chunk
    C[20_000:20_030] = C[7]                    # ... and in a middle chunk
    Q = np.concatenate([C[[7, 100, 300, 5000]], C[400:530] + rng.normal(0, 0.05, (130, L))])
    Q[1, :32] = 0.5                            # constant query segment
    corpus = IndexCorpus(C)
    qp = corpus.prepare_queries(Q)
    res = {}
    variants = {  # option settings of each variant (the default k_scan0g + k_sample_topg first)
        "v0": {},
        "v0-nosample": {"scan_nosample": 1},
        "v0-wpb4-pf3": {"scan_wpb": 4, "scan_pf": 3},
        "v0-pf4": {"scan_pf": 4},  # (the default scan is 3 waves per SIMD with 6 steps of prefetch)
        "v0-nb8": {"scan_nb": 8},  # 128-query waves
        "v0-occ4-pf4": {"scan_occ": 4, "scan_pf": 4},  # round 5's 4 waves per SIMD, 4096-wave geometry
        "v0-occ3-pf8": {"scan_occ": 3, "scan_pf": 8},
        "v0-occ3-pf4": {"scan_occ": 3, "scan_pf": 4},
        "v0-sample-full": {"sample_variant": 1},
        "v0-list": {"scan_variant": 1},  # k_scan0f
        "v1": {"scan_v1": 1},
    }
    for tag, opts in variants.items():
        for name in ("scan_nosample", "scan_wpb", "scan_pf", "scan_nb", "scan_occ", "sample_variant", "scan_variant",
                     "scan_v1"):
            hq_option(name, opts.get(name))
        for thr, tm in ((0.1, 1), (0.6, 1), (0.1, 2)):
            sc, ids, cnt, _, _ = corpus.exact_topk(qp, 0, 20, thr, tm)
            res[(tag, thr, tm)] = (_np(sc), _np(ids), _np(cnt))
        # M = 100 (a list of 108 > 64: every variant, scan_variant = 1 included, takes the queue scan)
        sc, ids, cnt, _, _ = corpus.exact_topk(qp, 0, 100, 0.1, 1)
        res[(tag, "m100", 1)] = (_np(sc), _np(ids), _np(cnt))
    for key in ((0.1, 1), (0.6, 1), (0.1, 2), ("m100", 1)):
        for tag in list(variants)[1:]:
            a, b = res[("v0",) + key], res[(tag,) + key]
            assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]), (tag, key)
            np.testing.assert_array_equal(a[0][a[1] >= 0], b[0][b[1] >= 0])
    s_ids, s_cnt = res[("v0", 0.1, 1)][1], res[("v0", 0.1, 1)][2]
    for a in list(range(6)) + [50, 133]:
        s = O.level_similarity(Q[a], C, 0)
        pos = np.nonzero(s >= 0.1)[0]
        ref = pos[np.argsort(-s[pos], kind="stable")][:20]
        assert list(s_ids[a][: s_cnt[a]]) == list(ref), a


@pytest.mark.parametrize("Q,N,K", [(3, 5, 4096), (130, 300, 1024), (257, 129, 1000), (64, 2000, 4096)])
def test_cosine_mfma_vs_f64(hq_lib, Q, N, K):
    """S7 on the matrix cores (split-f16 MFMA) == exact f64 cosine within 2e-6 on (cos + 1) / 2; zero rows
    give 0.0, mixed magnitudes and ragged tiles (Q, N not multiples of 128, K not of 32) included."""
    import torch
    from hq_mi355x import kernels as K_
    rng = np.random.default_rng(Q + N + K)
    A = (rng.standard_normal((Q, K)) * 10 ** rng.uniform(-3, 3, (Q, 1))).astype(np.float32)
    B = (rng.standard_normal((N, K)) * 10 ** rng.uniform(-3, 3, (N, 1))).astype(np.float32)
    B[: min(N, 4)] = A[0] * 2.0          # exact matches -> cos = 1
    A[-1] = 0.0                          # zero query row
    B[-1] = 0.0                          # zero frame row
    got = _np(K_.cosine_scores_mfma(K_.cos_prepare(torch.from_numpy(A).cuda()),
                                    K_.cos_prepare(torch.from_numpy(B).cuda())))
    a64, b64 = A.astype(np.float64), B.astype(np.float64)
    na, nb = np.linalg.norm(a64, axis=1), np.linalg.norm(b64, axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        want = ((a64 @ b64.T) / np.outer(na, nb) + 1.0) / 2.0
    want[na == 0, :] = 0.0
    want[:, nb == 0] = 0.0
    assert np.max(np.abs(got - want)) < 2e-6
    assert np.all(got[-1] == 0.0) and np.all(got[:, -1] == 0.0)


@pytest.mark.parametrize("Q,N,K", [(3, 5, 4096), (257, 129, 1000), (130, 700, 1024)])
def test_cosine_mfma_f32_scores(hq_lib, Q, N, K):
    """hq_cos_scores_mfma_f32: exactly the f64 scores rounded once to float32 (ragged tiles, zero rows)."""
    import torch
    from hq_mi355x import kernels as K_
    rng = np.random.default_rng(3 * Q + N + K)
    A = rng.standard_normal((Q, K)).astype(np.float32)
    B = rng.standard_normal((N, K)).astype(np.float32)
    A[-1] = 0.0
    pa, pb = K_.cos_prepare(torch.from_numpy(A).cuda()), K_.cos_prepare(torch.from_numpy(B).cuda())
    s64 = _np(K_.cosine_scores_mfma(pa, pb))
    s32 = _np(K_.cosine_scores_mfma(pa, pb, f32=True))
    assert s32.dtype == np.float32
    np.testing.assert_array_equal(s32, s64.astype(np.float32))


def test_cosine_mfma_vs_reference_golden(hq_lib, golden):
    """The reference's own float32 cosine values (rag/search/engine.py:622-660) within the north star's 1e-5."""
    import torch
    from hq_mi355x import kernels as K_
    g = golden("rag_score")
    A = g["cos_A"].reshape(len(g["cos_A"]), -1)
    B = g["cos_B"].reshape(1, -1)
    got = _np(K_.cosine_scores_mfma(K_.cos_prepare(torch.from_numpy(B).cuda()), K_.cos_prepare(torch.from_numpy(A).cuda())))[0]
    assert np.max(np.abs(got - g["cos"])) < 1e-5


@pytest.mark.parametrize("Q,N,K", [(130, 300, 1024), (257, 700, 4096), (1, 257, 32), (5, 40, 64)])
def test_cosine_dma_kernels_match_regstage(hq_lib, Q, N, K, hq_option):
    """The default tiled-layout kernel (k_cos_t<3, 1, 1>: 128 x 384 tiles, frame fragments straight into
    VGPRs one step ahead, query fragments through LDS, ping-pong wave groups), its other tile / prefetch /
    epilogue forms, the LDS-DMA ping-pong kernel (k_cos_g3<256, 1>: swizzled row-major LDS, staggered wave
    groups), its lockstep form and the register-staged baseline (k_cos_mfma, 128-frame tiles) run the same
    MFMA sequence per output, so their scores are bit-identical; ragged last frame tile (N not a multiple
    of 256) and 1- and 2-step K loops (K = 32, 64: the prologue / drain paths) included.  The layout of
    the prepared rows follows the kernel option, so each kernel prepares its own operands."""
    import torch
    from hq_mi355x import kernels as K_
    rng = np.random.default_rng(11 + Q + N)
    A = rng.standard_normal((Q, K)).astype(np.float32)
    B = rng.standard_normal((N, K)).astype(np.float32)

    def run():
        pa, pb = K_.cos_prepare(torch.from_numpy(A).cuda()), K_.cos_prepare(torch.from_numpy(B).cuda())
        return _np(K_.cosine_scores_mfma(pa, pb))
    got = run()
    for kern, code in (("tiled lockstep 128 x 256", 4), ("tiled 128 x 128", 5), ("tiled 128 x 256", 6),
                       ("tiled 128 x 256, one step ahead", 7), ("tiled, 16-byte stores", 8), ("ping-pong", 3),
                       ("lockstep", 2), ("regstage", 1)):
        hq_option("cos_kernel", code)
        np.testing.assert_array_equal(got, run(), err_msg=kern)


@pytest.mark.parametrize("L", [64, 32, 256])
def test_refine_rescore_equals_refine_then_rescore(hq_lib, hq_option, L):
    """hq_refine_rescore_topk (rows staged once in LDS, the re-score of the output from the same rows)
    returns exactly refine_topk's ranking plus hq_rescore's records for the output ids (zeros in empty
    slots), for the level-0 and the overall mode, on the LDS-staged and the global-memory kernels
    (L = 256 stages 97 KiB per query -> the global kernel + hq_rescore)."""
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    rng = np.random.default_rng(5 + L)
    N = 3000
    C = rng.standard_normal((N, L))
    C[10:14, : L // 2] = 0.5                   # constant level-0 segments
    C[40:45] = C[9]                            # duplicates (ties by id)
    Q = np.concatenate([C[[9, 10, 300]], C[500:560] + rng.normal(0, 0.05, (60, L))])
    corpus = IndexCorpus(C)
    qp = corpus.prepare_queries(Q)
    for mode, thr, tm in ((0, 0.1, 1), (1, 0.0, 0), (0, 0.97, 1)):
        if mode == 1 and not corpus._fused_ok(1):
            continue  # L = 256: the overall scan does not fuse (Lp > 256)
        asc, aid, _, _ = K.scan_topk(qp, corpus.prep, mode, 28, thr - corpus.EPS, 0 if tm == 0 else 1)
        for glob in (False, True):
            hq_option("refine_global", 1 if glob else None)
            s1, i1, c1, r1 = K.refine_topk(qp, corpus.prep, mode, asc, aid, 20, thr, tm, corpus.EPS)
            s2, i2, c2, r2, det = K.refine_rescore_topk(qp, corpus.prep, mode, asc, aid, 20, thr, tm, corpus.EPS)
            for x, y in ((s1, s2), (i1, i2), (c1, c2), (r1, r2)):
                np.testing.assert_array_equal(_np(x), _np(y), err_msg=f"mode {mode} thr {thr} global {glob}")
            ref = _np(K.rescore(qp, corpus.prep, i1))
            ids = _np(i1)
            ref[ids < 0] = 0.0
            np.testing.assert_array_equal(_np(det), ref, err_msg=f"mode {mode} thr {thr} global {glob}")
        assert (_np(c1) > 0).any()


@pytest.mark.parametrize("Q,N,k,thr,tm", [(3, 100_003, 20, 0.5, 1), (2, 70_000, 28, 0.0, 0), (5, 20_000, 10, 0.75, 2),
                                          (1, 8_193, 64, 0.0, 0)])
def test_two_stage_select_equals_one_stage(hq_lib, Q, N, k, thr, tm):
    """hq_select_topk_ws (parts of ~8192 entries in parallel, then a merge in the same total order) gives the
    one-stage hq_select_topk's top-k, ids and first arg-max exactly, with heavy ties (scores on a coarse
    grid), entries below the threshold and rows where fewer than k entries pass."""
    import torch
    from hq_mi355x import _lib, kernels as K
    from hq_mi355x._dev import ptr, stream
    rng = np.random.default_rng(Q * 7 + k)
    sc = np.round(rng.random((Q, N)), 2)       # ties everywhere
    sc[0, N // 3] = 2.0                        # unique maximum in a middle part
    if Q > 1:
        sc[1, :] = np.minimum(sc[1, :], thr)   # nothing (or everything at thr) passes in row 1
    S = _t(sc)
    a = K.select_topk(S, k, thr, tm, 5)
    os_ = torch.empty((Q, k), dtype=torch.float64, device=S.device)
    oi = torch.empty((Q, k), dtype=torch.int64, device=S.device)
    b = torch.empty(Q, dtype=torch.float64, device=S.device)
    bi = torch.empty(Q, dtype=torch.int64, device=S.device)
    _lib.check(_lib.lib().hq_select_topk(ptr(S), Q, N, k, float(thr), tm, 5, ptr(os_), ptr(oi), ptr(b), ptr(bi),
                                         stream()))
    for x, y in zip(a, (os_, oi, b, bi)):
        np.testing.assert_array_equal(_np(x), _np(y))
    ok = sc >= thr if tm == 1 else (sc > thr if tm == 2 else np.ones_like(sc, bool))
    for q in range(Q):
        pos = np.nonzero(ok[q])[0]
        ref = pos[np.lexsort((pos, -sc[q, pos]))][:k] + 5
        got = _np(a[1])[q]
        assert list(got[got >= 0]) == list(ref)


def test_statistical_start_threshold_is_exact(hq_lib, hq_option):
    """A starting threshold from the sample's K'-th best (K' < K; the default is 12 on sparse samples) is not
    a provable bound: lists left short are marked (+inf in the empty slots) and their queries answered by
    the dense exact path.  With K' = 1 most lists are short; the progressive results must equal the
    provable mode's (option sample_kth = 0) and the oracle's."""
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    rng = np.random.default_rng(31)
    N, L = 70_000, 64                           # sample stride 17: the statistical threshold applies
    C = rng.standard_normal((N, L))
    C[500:520] = C[77]                          # duplicates of a query row
    Q = np.concatenate([C[[77, 5, 9000]], C[100:140] + rng.normal(0, 0.05, (40, L))])
    corpus = IndexCorpus(C)
    out = {}
    for kth in ("0", "16", "1"):
        hq_option("sample_kth", int(kth))
        ids, ov, lv, cnt = corpus.progressive(Q, 10, 0.1, 20)
        out[kth] = (_np(ids), _np(ov), _np(lv), _np(cnt))
        if kth == "1":
            qp = corpus.prepare_queries(Q)
            asc, aid, _, _ = K.scan_topk(qp, corpus.prep, 0, 28, 0.1 - corpus.EPS, 1)
            _, _, _, res = K.refine_topk(qp, corpus.prep, 0, asc, aid, 20, 0.1, 1, corpus.EPS)
            trunc = (_np(aid)[:, -1] < 0) & (_np(asc)[:, -1] == np.inf)
            assert trunc.any() and not _np(res)[trunc].any()
    for kth in ("16", "1"):
        for x, y in zip(out["0"], out[kth]):
            np.testing.assert_array_equal(x, y, err_msg=kth)
    ids, cnt = out["1"][0], out["1"][3]
    for a in (0, 1, 20):
        rid, _, _, _ = O.progressive_search(Q[a], C, 10, 0.1, 20)
        assert list(ids[a][: cnt[a]]) == list(rid), a


def _np_select(row, k, thr, thr_mode):
    """Reference of hq_select_topk: top-k by (score desc, index asc) among entries passing the
    threshold test, padded with (-inf, -1); first arg-max over all entries."""
    idx = np.arange(len(row))
    ok = np.ones(len(row), bool) if thr_mode == 0 else (row >= thr if thr_mode == 1 else row > thr)
    cand = sorted(zip(-row[ok], idx[ok]))[:k]
    s = [-a for a, _ in cand] + [-np.inf] * (k - len(cand))
    i = [b for _, b in cand] + [-1] * (k - len(cand))
    b = min(zip(-row, idx))
    return np.array(s), np.array(i), -b[0], b[1]


@pytest.mark.parametrize("N", [1, 100, 1025, 9000, 70000])
def test_select_topk_register_stages(hq_lib, hq_option, N):
    """The register-resident multi-stage select (few queries: the dense redo) equals the reference order
    and the two-stage select, with ties (quantised scores), thresholds and id_base."""
    import torch
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(N)
    sc = np.round(rng.random((3, N)), 2)  # many ties
    for k in (16, 20, 28, 64):
        for thr, mode in ((0.0, 0), (0.5, 1), (0.5, 2), (0.995, 1)):
            got = [_np(x) for x in K.select_topk(torch.tensor(sc, device="cuda"), k, thr, mode, 7)]
            hq_option("select_2stage", 1)
            two = [_np(x) for x in K.select_topk(torch.tensor(sc, device="cuda"), k, thr, mode, 7)]
            hq_option("select_2stage", None)
            for x, y in zip(got, two):
                assert np.array_equal(x, y), (N, k, thr, mode)
            for q in range(3):
                s, i, b, bi = _np_select(sc[q], k, thr, mode)
                assert np.array_equal(got[0][q], s) and np.array_equal(got[1][q], np.where(i >= 0, i + 7, -1)), (N, k, q)
                assert got[2][q] == b and got[3][q] == bi + 7


def test_rccl_allgather_one_rank(hq_lib):
    """hq_allgather_topk on a one-rank RCCL communicator (hq_comm_init_rank): recv == send, [1, ...] shaped,
    for the record layout of the sharded search and an odd byte count."""
    import torch
    from hq_mi355x.rccl import Communicator
    comm = Communicator.single()
    assert (comm.nranks, comm.rank) == (1, 0)
    x = torch.randn((1000, 21, 8), dtype=torch.float64, device="cuda")
    y = comm.all_gather(x)
    assert y.shape == (1,) + tuple(x.shape) and torch.equal(y[0], x)
    b = torch.arange(37, dtype=torch.uint8, device="cuda")
    assert torch.equal(comm.all_gather(b)[0], b)
    comm.close()


def test_rag_spatial_locality_enhanced_golden(hq_lib, golden):
    """S7 completed: _calculate_spatial_locality_similarity through _extract_original_embedding (original
    height detected on each enhanced image: the RAG generator's index rows cut off, rag/search/engine.py:
    134-162, 604-714) against the reference's own values, float32 AND float64 images (float64 kept in
    float64), batched Q x N on the GPU (hq_spatial_locality) and as the pairwise drop-in."""
    from hq_mi355x.rag import similarity as S
    g = golden("rag_score")
    for tag in ("s64f", "s64d", "s32f", "s8d"):
        enh = g[f"{tag}_enh"]
        tol = 1e-6 if enh.dtype == np.float32 else 1e-12
        assert list(S.detect_original_embedding_heights(enh)) == list(g[f"{tag}_heights"]), tag
        got = _np(S.spatial_locality_scores(enh[:2], enh))
        np.testing.assert_allclose(got, g[f"{tag}_spatial"], atol=tol, err_msg=tag)
        assert abs(S.calculate_spatial_locality_similarity(enh[0], enh[1]) - g[f"{tag}_spatial"][0, 1]) < tol
        ex = S.extract_original_embedding(enh[0])
        assert ex.shape == (g[f"{tag}_heights"][0], enh.shape[2]) and ex.dtype == enh.dtype
    t = g["tiny_enh"]
    assert abs(S.calculate_spatial_locality_similarity(t[0], t[1]) - g["tiny_spatial"][0]) < 1e-12


def test_rag_progressive_threshold_golden(hq_lib, golden):
    """S7 completed: _apply_progressive_threshold (rag/search/engine.py:243-287) as a device select
    (hq_threshold_select): level thresholds 0.6 / 0.5 / 0.4 / 0.3 (Python float sums, scores placed on
    them), caps 30 / 50 / 70 % of the list, candidate order kept; batched rows agree with the drop-in."""
    from hq_mi355x.rag import similarity as S
    g = golden("rag_score")
    sc, ids = g["thr_scores"], g["thr_ids"]
    for level in range(5):
        for cut in (200, 37, 1):
            got = S.apply_progressive_threshold(list(zip(ids[:cut].tolist(), sc[:cut].tolist())), level)
            ref = g[f"thr_l{level}_n{cut}"]
            assert got == list(ref[ref >= 0]), (level, cut)
        rows = np.stack([sc, sc[::-1]])
        out, cnt = S.progressive_threshold_batch(rows, level)
        out, cnt = _np(out), _np(cnt)
        for r in range(2):
            want = O.rag_progressive_threshold(list(enumerate(rows[r].tolist())), level)
            assert list(out[r][: cnt[r]]) == want and np.all(out[r][cnt[r]:] == -1)


def test_rag_cosine_float64_kept(hq_lib):
    """float64 embeddings are scored in float64 (no narrowing to float32): the drop-in cosine equals the
    f64 oracle to 1e-14 on values whose float32 rounding alone would move the score by > 1e-9."""
    from hq_mi355x.rag import similarity as S
    rng = np.random.default_rng(3)
    a = 1.0 + rng.standard_normal(4096) * 1e-7
    b = 1.0 + rng.standard_normal(4096) * 1e-7
    want = float(O.rag_cosine(a, b[None])[0])
    assert abs(S.calculate_embedding_cosine_similarity(a, b) - want) < 1e-14
    A = rng.standard_normal((5, 3, 64))
    got = [S.compare_multi_level_indices(A[0], A[i]) for i in range(5)]
    np.testing.assert_allclose(got, O.rag_multi_level_similarity(A[0], A), atol=1e-14)


@pytest.mark.parametrize("N,L", [(70_003, 64), (3_001, 64), (20_000, 32)])
def test_overall_split_scan_matches_f64_scan(hq_lib, hq_option, N, L):
    """The split-f16 overall scan (hq_scanov_topk_split: segment-packed contractions, pre-filter bound,
    pools) + exact re-rank gives the same brute-force top-k as the f64 k_scan (option scan_v1) and as the
    oracle, and leaves (almost) every query resolved: corpus with zero-variance segments, duplicates, and
    one-value segments equal to / within 1e-6 of / just past 1e-6 from the query's."""
    from hq_mi355x import kernels as K_
    from hq_mi355x.core.search_engine import IndexCorpus
    rng = np.random.default_rng(N + L)
    C = rng.standard_normal((N, L))
    segs = O.segment_bounds(L)
    one = [s for s, e in segs if e - s == 1]
    s1, e1 = segs[1]
    C[::7, s1:e1] = 0.25                           # zero-variance segment on every 7th row
    C[N // 2: N // 2 + 40] = C[11]                  # duplicates
    Q = np.concatenate([C[[11, 12, 13, 500]] + 0.0, C[1000:1100] + rng.normal(0, 0.01, (100, L))])
    Q[2, s1:e1] = 0.25                             # zero-variance query segment (both-constant pairs)
    for o in one:                                  # one-value segments: equal, 5e-7 apart, 2e-6 apart
        C[20:40, o] = Q[0, o]
        C[40:60, o] = Q[0, o] + 5e-7
        C[60:80, o] = Q[0, o] + 2e-6
    corpus = IndexCorpus(C)
    assert corpus.prep.Zov16 is not None
    qp = corpus.prepare_queries(Q)
    k = 10
    got = [_np(x) for x in corpus.exact_topk(qp, 1, k)[:3]]
    sc, ids, _, _ = K_.scan_topk(qp, corpus.prep, 1, k + corpus.SLACK, -corpus.EPS, 0)
    _, _, _, res = K_.refine_topk(qp, corpus.prep, 1, sc, ids, k, 0.0, 0, corpus.EPS)
    assert int(_np(res).sum()) >= len(Q) - 2        # the dense fallback stays an exception
    hq_option("ov_occ", 3)                         # the 3-waves-per-SIMD build of k_scanov
    occ3 = [_np(x) for x in corpus.exact_topk(qp, 1, k)[:3]]
    assert np.array_equal(got[1], occ3[1]) and np.array_equal(got[0], occ3[0])
    hq_option("ov_occ", None)
    hq_option("scan_v1", 1)
    ref = [_np(x) for x in corpus.exact_topk(qp, 1, k)[:3]]
    assert np.array_equal(got[1], ref[1]) and np.array_equal(got[0], ref[0])
    for a in (0, 1, 2, 3, 50):
        rid, rsc, _ = O.brute_force_search(Q[a], C, k)
        assert list(got[1][a]) == list(rid), a
        np.testing.assert_allclose(got[0][a], rsc, atol=TOL)


def test_dropin_pool_corpus_reused_per_pool(hq_lib):
    """ProgressiveSimilaritySearchEngine keeps the resident corpus of the last uniform pool: the same
    pool (same index arrays, same order) re-uses it; a pool with one model replaced, or re-ordered, is
    re-uploaded, and every call still equals the oracle."""
    from hq_mi355x.core import ProgressiveSimilaritySearchEngine
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    C = _corpus(400, 64, 21)
    pool = [QuantizedModel(b"x", (8, 8), 1, 0.8, C[i], ModelMetadata(f"m{i}", 1, 1, 1.0, "t")) for i in range(len(C))]
    eng = ProgressiveSimilaritySearchEngine(0.1, 20)
    rng = np.random.default_rng(5)

    def check(p, q):
        r = eng.brute_force_search(q, p, 10)
        M = np.stack([m.hierarchical_indices for m in p])
        rid, rsc, _ = O.brute_force_search(q, M, 10)
        pos = {id(m): i for i, m in enumerate(p)}
        assert [pos[id(x.model)] for x in r] == list(rid)

    q = C[7] + rng.normal(0, 0.01, 64)
    check(pool, q)
    first = eng._pool_cache[1]
    check(pool, C[9] + 0.0)
    assert eng._pool_cache[1] is first                        # same pool: no re-upload
    pool2 = list(pool)
    pool2[3] = QuantizedModel(b"x", (8, 8), 1, 0.8, C[7] + 1e-3, ModelMetadata("new", 1, 1, 1.0, "t"))
    check(pool2, q)
    assert eng._pool_cache[1] is not first                    # a replaced model: new corpus
    check(pool2[::-1], q)                                     # re-ordered: new corpus, ids follow the order
