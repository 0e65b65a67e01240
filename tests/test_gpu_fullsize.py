"""Parity at the BASELINE full sizes (cfg2 1M x 1536, cfg3 1M-row corpus x 1000 queries, cfg5 7e9 f16
values, the S7 bench shape).  The oracle cannot run these sizes in seconds, so every row is checked
through size-independent properties (min/max of each quantized image, the 0 / 255 end points of every
frame, self-matches, score ranges and order) and a seeded sample of rows is checked bit-exact (or
within the stated tolerance) against the oracle."""
import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def _sample(n, k, seed):
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, k)]))


def _oracle_many(Qh, Ch, rows):
    """oracle.progressive_search (top-10 of M = 20, threshold 0.1) for the sampled query rows on 8 host
    threads (the vectorised oracle spends its time in NumPy calls that release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda a: O.progressive_search(Qh[a], Ch, 10, 0.1, 20), rows))


def test_cfg2_full_size(hq_lib):
    """cfg2: 1M x 1536 f32, order-64 map + streaming index (L = 64) + embed + u8 (fused kernel)."""
    import torch
    from hq_mi355x import kernels as K
    N, d, n, L = 1_000_000, 1536, 64, 64
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn((N, d), generator=g, device="cuda", dtype=torch.float32)
    fr, idx, mm = K.map_index_quantize(X, n, L)
    torch.cuda.synchronize()
    # the enhanced image holds the data, the zero padding (d < n^2) and means of both, so its
    # min / max are those of the data and 0
    assert torch.equal(mm[:, 0], torch.clamp(X.min(1).values, max=0.0))
    assert torch.equal(mm[:, 1], torch.clamp(X.max(1).values, min=0.0))
    # every (non-constant) frame spans 0 .. 255: trunc((v - mn) / (mx - mn) * 255) at mn and mx
    flat = fr.view(N, -1)
    assert int(flat.min(1).values.max()) == 0 and int(flat.max(1).values.min()) == 255
    # the first index value is level 0 at position 0: the first parameter
    assert torch.equal(idx[:, 0], X[:, 0].double())
    rows = _sample(N, 300, 11)
    P = _np(X[torch.from_numpy(rows).cuda()])
    F, I, M = _np(fr[torch.from_numpy(rows).cuda()]), _np(idx[torch.from_numpy(rows).cuda()]), \
        _np(mm[torch.from_numpy(rows).cuda()])
    for r in range(len(rows)):
        img = O.map_to_2d(O.pad_parameters(P[r], n), n)
        ridx = O.streaming_index(O.map_from_2d(img), L)
        u8, mn, mx = O.normalize_u8(O.embed_index_row(img, ridx))
        assert F[r].tobytes() == u8.tobytes(), rows[r]
        assert I[r].tobytes() == ridx.tobytes(), rows[r]
        assert M[r, 0] == mn and M[r, 1] == mx


def test_cfg5_full_size(hq_lib):
    """cfg5: 7e9 f16 values in 1024-value chunks (6,835,938 chunks; the 512-value tail chunk maps to
    32 x 32 at efficiency 0.5), traditional index (L = 32), u8 frames."""
    import torch
    from hq_mi355x import kernels as K
    total = 7_000_000_000
    nfull = total // 1024
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn((total,), generator=g, device="cuda", dtype=torch.float16).mul_(0.02)
    fr, idx, mm = K.chunk_encode_f16(x, 1024)
    torch.cuda.synchronize()
    assert fr.shape[0] == nfull + 1
    xv = x[: nfull * 1024].view(nfull, 1024)
    # full chunks: the index row ends in zeros (16 means + 10 samples + 6 zeros at L = 32), so the
    # frame's min / max are those of the chunk and 0
    assert torch.equal(mm[:nfull, 0], torch.clamp(xv.min(1).values.float(), max=0.0))
    assert torch.equal(mm[:nfull, 1], torch.clamp(xv.max(1).values.float(), min=0.0))
    flat = fr[:nfull].view(nfull, -1)
    const = mm[:nfull, 0] == mm[:nfull, 1]
    assert int(flat.min(1).values[~const].max()) == 0 and int(flat.max(1).values[~const].min()) == 255
    rows = np.concatenate([_sample(nfull, 200, 12), [nfull]])   # + the 512-value tail chunk
    xs = _np(x)  # host copy for the sampled chunks (14 GB of f16 on the box's host memory is fine)
    F, I, M = _np(fr), _np(idx), _np(mm)
    for c in rows:
        ch = xs[c * 1024:(c + 1) * 1024].astype(np.float32)
        m = O.optimal_dimensions(len(ch))[0]
        img = O.map_to_2d(ch, m)
        ridx = O.traditional_index(img, m)
        u8, mn, mx = O.normalize_u8(O.embed_index_row(img, ridx))
        assert F[c][: m + 1, :m].tobytes() == u8.tobytes(), c
        assert I[c][:m].tobytes() == ridx.tobytes(), c
        assert M[c, 0] == mn and M[c, 1] == mx


def test_cfg3_full_size(hq_lib):
    """cfg3: progressive top-10 over a 1M-row corpus (L = 64 index vectors of seed-2 embeddings from the
    fused kernel), 1000 queries = corpus rows 0..999 + N(0, 0.01) noise (the bench's workload)."""
    import torch
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    N, Qn = 1_000_000, 1000
    g = torch.Generator(device="cuda").manual_seed(2)
    Xc = torch.randn((N, 1536), generator=g, device="cuda", dtype=torch.float32)
    _, C, _ = K.map_index_quantize(Xc, 64, 64)
    del Xc
    gq = torch.Generator(device="cuda").manual_seed(3)
    Q = C[:Qn] + 0.01 * torch.randn((Qn, 64), generator=gq, device="cuda", dtype=torch.float64)
    ids, ov, lv, cnt = IndexCorpus(C).progressive(Q, 10, 0.1, 20)
    ids, ov, cnt = _np(ids), _np(ov), _np(cnt)
    assert np.array_equal(ids[:, 0], np.arange(Qn))            # every query finds its own row first
    assert np.all(cnt == 10)
    assert np.all((ov >= 0.0) & (ov <= 1.0)) and np.all(np.diff(ov, axis=1) <= 0.0)
    Ch, Qh = _np(C), _np(Q)
    sample = _sample(Qn, 22, 31).tolist()
    for a, (rid, rsc, _, _) in zip(sample, _oracle_many(Qh, Ch, sample)):
        assert list(ids[a]) == list(rid), a
        np.testing.assert_allclose(ov[a], rsc, atol=1e-10)  # as test_gpu_search.TOL


def test_frames_bench_shape(hq_lib):
    """S7 at the bench shape: 1000 query frames x 250k stored 64 x 64 frames; queries 0..999 are copies
    of stored frames, so their own score is the row maximum (cos = 1); sampled rows vs an f64 cosine
    within the north star's 1e-5 (measured < 2e-6)."""
    import torch
    from hq_mi355x import kernels as K
    Nf, Qn, Kd = 250_000, 1000, 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    F = torch.randn((Nf, Kd), generator=g, device="cuda", dtype=torch.float32)
    S = K.cosine_scores_mfma(K.cos_prepare(F[:Qn].clone()), K.cos_prepare(F))
    torch.cuda.synchronize()
    # (cos + 1) / 2 is not clamped (rag/search/engine.py:657-660): rounding may pass 0 or 1 by < 2e-6
    assert bool(((S >= -2e-6) & (S <= 1.0 + 2e-6)).all())
    own = S[torch.arange(Qn, device="cuda"), torch.arange(Qn, device="cuda")]
    assert float((1.0 - own).abs().max()) < 2e-6
    assert torch.equal(S.argmax(1).cpu(), torch.arange(Qn))
    cols = torch.from_numpy(_sample(Nf, 20000, 13)).cuda()
    B = _np(F[cols]).astype(np.float64)
    nb = np.linalg.norm(B, axis=1)
    for q in (0, 421, 999):
        a = _np(F[q]).astype(np.float64)
        want = (B @ a / (nb * np.linalg.norm(a)) + 1.0) / 2.0
        got = _np(S[q, cols])
        assert np.max(np.abs(got - want)) < 2e-6, q


def test_cfg4_full_size_8_shards(hq_lib):
    """cfg4 on one GPU: the 8M-row corpus (L = 64 index vectors of seed-4 embeddings from the fused kernel,
    generated 1M rows at a time) as 8 ShardedIndexCorpus shards of 1M rows, each answering the cfg3-style
    1000-query batch (global rows 0..999 + N(0, 0.01) noise, seed 3); the records merged by
    ShardedIndexCorpus.merge (hq_progressive_final, 8-way) == an unsharded IndexCorpus over all 8M rows:
    ids, counts, overall and per-level scores bit-identical; sampled queries == the oracle
    (core/search_engine.py:232-300, 340-388; merge analogue core/video_search.py:722-875).  One shard also
    runs its all-gather through a one-rank RCCL communicator (hq_allgather_topk)."""
    import torch
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus, shard_range
    from hq_mi355x.rccl import Communicator
    R, per, Qn = 8, 1_000_000, 1000
    N = R * per
    g = torch.Generator(device="cuda").manual_seed(4)
    C = torch.empty((N, 64), dtype=torch.float64, device="cuda")
    for r in range(R):
        Xc = torch.randn((per, 1536), generator=g, device="cuda", dtype=torch.float32)
        _, C[r * per:(r + 1) * per], _ = K.map_index_quantize(Xc, 64, 64)
        del Xc
    gq = torch.Generator(device="cuda").manual_seed(3)
    Q = C[:Qn] + 0.01 * torch.randn((Qn, 64), generator=gq, device="cuda", dtype=torch.float64)
    full = IndexCorpus(C)
    ref = [_np(x) for x in full.progressive(Q, 10, 0.1, 20)]
    del full
    recs = []
    for r in range(R):
        a, b = shard_range(N, r, R)
        sh = ShardedIndexCorpus(C[a:b], id_base=a, n_total=N)
        recs.append(sh.local_records(sh.local.prepare_queries(Q), 20, 0.1))
        del sh
    oid, ov, lv, cnt = ShardedIndexCorpus.merge(torch.stack(recs, 0), 20, 10)
    for x, y, name in zip((oid, ov, lv, cnt), ref, ("ids", "overall", "levels", "count")):
        np.testing.assert_array_equal(_np(x), y, err_msg=name)
    ids = ref[0]
    assert np.array_equal(ids[:, 0], np.arange(Qn)) and np.all(ref[3] == 10)
    # the C-ABI all-gather on a one-rank communicator: the sharded path end to end (shard = whole corpus)
    comm = Communicator.single()
    one = ShardedIndexCorpus(C[:per], id_base=0, n_total=per, comm=comm)
    got = [_np(x) for x in one.progressive(Q, 10, 0.1, 20)]
    want = [_np(x) for x in IndexCorpus(C[:per]).progressive(Q, 10, 0.1, 20)]
    for x, y in zip(got, want):
        np.testing.assert_array_equal(x, y)
    comm.close()
    Ch, Qh = _np(C), _np(Q)
    sample = sorted(set([333] + _sample(Qn, 5, 41).tolist()))
    for a, (rid, rsc, _, _) in zip(sample, _oracle_many(Qh, Ch, sample)):
        assert list(ids[a]) == list(rid), a
        np.testing.assert_allclose(ref[1][a], rsc, atol=1e-10)
