"""World-size-2 rehearsal of the corpus-sharded search protocol on CPU with gloo.

Each rank holds a contiguous shard (hq_mi355x.distributed.shard_range), computes what its GPU would
compute — the exact level-0 top-M >= threshold of its shard, its first arg-max, and the exact overall /
per-level re-scores — here with the oracle, packs the records (distributed.pack), exchanges them with
the real all-gather helper (distributed.all_gather, one collective), unpacks them and merges with the
rule hq_progressive_final implements on the GPU: global top-M by (level-0 score desc, global id asc),
the first arg-max when nothing passed, then a stable sort by the overall score.  The merged result must
equal the oracle's progressive search over the whole corpus.  (The GPU merge kernel itself is checked
against the unsharded scan in tests/test_gpu_search.py::test_sharded_merge_equals_single.)
"""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import hq_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus():
    rng = np.random.default_rng(21)
    C = rng.standard_normal((401, 64)).cumsum(1) * 0.1
    C[300:305] = C[17]        # duplicates in the other shard: ties must follow global ids
    C[40, :32] = 0.5          # zero-variance level-0 segment
    Q = np.concatenate([C[[17, 250, 40]], C[100:104] + rng.normal(0, 0.02, (4, 64))])
    return C, Q


def _local_records(q, shard, base, M, thr):
    """One rank's contribution for query q: M slots of [s0, gid, overall, levels...] + best slot."""
    s = O.level_similarity(q, shard, 0)
    pos = np.nonzero(s >= thr)[0]
    pos = pos[np.argsort(-s[pos], kind="stable")][:M]
    nlev = len(O.parse_index_structure(len(q)))
    W = 1 + nlev
    rec = np.zeros((M + 1, 2 + W))
    rec[:, 0] = -np.inf
    rec[:, 1] = -1
    if len(pos):
        ov, per = O.overall_similarity(q, shard[pos])
        rec[: len(pos), 0] = s[pos]
        rec[: len(pos), 1] = pos + base
        rec[: len(pos), 2] = ov
        rec[: len(pos), 3:] = per
    b = int(np.argmax(s))
    ov, per = O.overall_similarity(q, shard[[b]])
    rec[M, 0], rec[M, 1], rec[M, 2], rec[M, 3:] = s[b], b + base, ov[0], per[0]
    return rec


def _merge(g, M, K):
    """hq_progressive_final's rule on gathered records g [R, M + 1, 2 + W] of one query."""
    R = g.shape[0]
    cand = [(g[r, i, 0], int(g[r, i, 1]), r, i) for r in range(R) for i in range(M) if g[r, i, 1] >= 0]
    cand.sort(key=lambda x: (-x[0], x[1]))
    surv = cand[:M]
    if not surv:
        best = max(((g[r, M, 0], -int(g[r, M, 1]), r) for r in range(R)))
        r = best[2]
        rows = [g[r, M]]
    else:
        rows = [g[r, i] for (_, _, r, i) in surv]
    order = sorted(range(len(rows)), key=lambda i: -rows[i][2])  # stable by overall
    rows = [rows[i] for i in order][:K]
    return [int(x[1]) for x in rows], [x[2] for x in rows]


def _worker(rank, world, port, out_path, M, K, thr):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
    import torch.distributed as dist
    from hq_mi355x import distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C, Q = _corpus()
        a, b = D.shard_range(len(C), rank, world)
        recs = np.stack([_local_records(q, C[a:b], a, M, thr) for q in Q])  # [Q, M + 1, 2 + W]
        t = torch.from_numpy(recs)
        s, ids, det = D.unpack(t)
        packed = D.pack(s, ids, det)                  # the GPU path's record layout round trip
        assert torch.equal(packed, t)
        g = D.all_gather(packed)                      # [R, Q, M + 1, 2 + W]
        if rank == 0:
            res = [_merge(g[:, qi].numpy(), M, K) for qi in range(len(Q))]
            np.save(out_path, np.array([r[0] + [-1] * (K - len(r[0])) for r in res]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("thr", [0.1, 0.99])
def test_sharded_protocol_world2_gloo(thr):
    M, K, world = 20, 10, 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ids.npy")
        mp.spawn(_worker, args=(world, _free_port(), out, M, K, thr), nprocs=world, join=True)
        got = np.load(out)
    C, Q = _corpus()
    for qi, q in enumerate(Q):
        rid, _, _, _ = O.progressive_search(q, C, K, thr, M)
        assert list(got[qi][: len(rid)]) == list(rid), (qi, got[qi], rid)


def test_shard_ranges_cover():
    from hq_mi355x.distributed import shard_range
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1
