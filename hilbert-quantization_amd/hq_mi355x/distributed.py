"""Corpus sharding across GPUs: one process per GPU, the corpus split into contiguous
global-id ranges, every rank answering the whole query batch against its shard, and ONE all-gather
(torch.distributed, backend "nccl" = RCCL over xGMI) of fixed-size per-shard records, merged on
every rank by the same (score desc, global id asc) rule that reproduces the single-GPU order.

The reference has no distributed component; its closest analogue is the per-video thread fan-out
plus list-concatenation merge of core/video_search.py:722-875.

Record layout per (query, slot), float64: [score, id, det_0 .. det_{W-1}] where det = [overall,
level sims...] from hq_rescore; ids are integers < 2^53 so the f64 round trip is exact.
"""
from __future__ import annotations

from typing import Optional, Tuple

from . import kernels as K
from ._dev import torch
from .core.search_engine import IndexCorpus


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, end) global-id range of a rank (balanced, ranks in order)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack(scores, ids, det):
    """[Q, M] scores, [Q, M] ids, [Q, M, W] det -> f64 [Q, M, 2 + W] records."""
    t = torch()
    return t.cat([scores.unsqueeze(-1).to(t.float64), ids.unsqueeze(-1).to(t.float64), det.to(t.float64)], dim=-1)


def unpack(rec):
    """[..., 2 + W] records -> (scores, ids int64, det)."""
    t = torch()
    return rec[..., 0].contiguous(), rec[..., 1].round().to(t.int64).contiguous(), rec[..., 2:].contiguous()


def all_gather(x, group=None, comm=None):
    """Stack of every rank's tensor [R, ...] (one collective).  comm (rccl.Communicator): RCCL through the
    C-ABI (hq_allgather_topk); else torch.distributed on `group` (RCCL on GPU tensors, gloo on CPU)."""
    if comm is not None:
        return comm.all_gather(x)
    t = torch()
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return x.unsqueeze(0)
    world = dist.get_world_size(group)
    out = [t.empty_like(x) for _ in range(world)]
    dist.all_gather(out, x.contiguous(), group=group)
    return t.stack(out, 0)


class ShardedIndexCorpus:
    """This rank's shard of a global corpus of index vectors (global ids start at `id_base`)."""

    def __init__(self, local_indices, id_base: int, n_total: int, group=None, comm=None):
        """comm: an rccl.Communicator over the shard ranks (the C-ABI all-gather); without it the records
        travel by torch.distributed.all_gather on `group`."""
        self.local = IndexCorpus(local_indices, id_base=id_base)
        self.n_total = int(n_total)
        self.group = group
        self.comm = comm

    def local_records(self, qp, M: int, threshold: float):
        """This shard's exact contribution [Q, M + 1, 2 + W]: the level-0 top-M >= threshold by (score
        desc, global id asc) with exact overall / level re-scores, plus the shard's first arg-max slot
        (used only when no shard has a passing candidate).  The scan, re-rank, re-scores and packing
        are queued before the one host sync, which only checks for rows that need the dense exact path
        (list not proven complete, or nothing passed -> arg-max)."""
        return self._local_finish(self._local_submit(qp, M, threshold))

    def _local_submit(self, qp, M: int, threshold: float):
        """Queue the shard's records; the redo flag leaves for pinned host memory behind them."""
        t = torch()
        c = self.local
        Q = qp.N
        slack = c.slack_for(M)
        s0, ids, cnt, res, det0 = c._scan_refine(qp, 0, M, float(threshold), 1, det=True, slack=slack)
        # no arg-max on the scan path (count-0 rows are redone below): constant fallback slot
        best, bid, bdet0 = c._no_fallback(Q, qp.Z.device)
        rec = self._records(qp, s0, ids, best, bid, det0, bdet0.view(Q, 1, -1))
        redo = (res == 0) | (cnt == 0)
        forced = c._forced(qp)
        if forced is not None:
            redo = redo | forced
        flag = c._pinned(t.bool)
        flag.copy_(redo.any().view(1), non_blocking=True)
        ev = t.cuda.Event()
        ev.record()
        return qp, M, float(threshold), rec, (redo, res, cnt, forced, M + slack), flag, ev

    def _local_finish(self, pending):
        t = torch()
        qp, M, threshold, rec, (redo, res, cnt, forced, kp), flag, ev = pending
        ev.synchronize()
        any_redo = bool(flag[0])
        self.local._unpin(flag)  # read: reusable
        if any_redo:
            # unproven lists re-scanned with a longer list, the rest on the dense exact path (IndexCorpus)
            sel = t.nonzero(redo).view(-1)
            s2, i2, b2, bi2, d2, bd2 = self.local._level0_redo(qp, sel, M, threshold, res, cnt, forced, kp=kp)
            rec[sel] = self._records(qp.rows(sel), s2, i2, b2, bi2, d2, bd2.view(-1, 1, bd2.shape[-1]))
        return rec

    def _records(self, q, s0_, ids_, best_, bid_, det=None, bdet=None):
        t = torch()
        c = self.local
        if det is None:
            det = K.rescore(q, c.prep, ids_, c.id_base)
        if bdet is None:
            bdet = K.rescore(q, c.prep, bid_.view(-1, 1), c.id_base)
        return t.cat([pack(s0_, ids_, det), pack(best_.view(-1, 1), bid_.view(-1, 1), bdet)], dim=1)

    @staticmethod
    def merge(g, M: int, max_results: int, key32: bool = False):
        """Merge gathered records [R, Q, M + 1, 2 + W] exactly as the single-GPU ranking (key32: every
        vector float32, IndexCorpus.key32)."""
        gs, gi, gd = unpack(g[:, :, :M])
        bs, bi, bd = unpack(g[:, :, M])
        oid, odet, cnt = K.progressive_final(gs, gi, gd, bs, bi, bd, int(max_results), key32=key32)
        return oid, odet[..., 0], odet[..., 1:], cnt

    def progressive(self, queries, max_results: int, threshold: float = 0.1, max_candidates_per_level: int = 100):
        """Global progressive search; every rank returns the same (ids, overall, levels, count)."""
        return self.progressive_finish(self.progressive_submit(queries, max_results, threshold,
                                                               max_candidates_per_level))

    def progressive_submit(self, queries, max_results: int, threshold: float = 0.1,
                           max_candidates_per_level: int = 100):
        """Queue this shard's part of a global progressive search (IndexCorpus.progressive_submit); the
        all-gather and merge run in progressive_finish, which every rank calls in the same batch order."""
        c = self.local
        M = int(max_candidates_per_level)
        if self.n_total <= M:
            return ["done", self.brute_force(queries, max_results)]
        qp = c.prepare_queries(queries)
        if M + c.SLACK > c._max_list(0) or c.dense_only or not c._fused_ok(0):  # the dense exact path per shard (list length / f32 model)
            t = torch()
            Q = qp.N
            s0, ids, _, best, bid = c.exact_topk(qp, 0, M, float(threshold), 1, need_best=True)
            det = K.rescore(qp, c.prep, ids, c.id_base)
            bdet = K.rescore(qp, c.prep, bid.view(Q, 1), c.id_base)
            rec = t.cat([pack(s0, ids, det), pack(best.view(Q, 1), bid.view(Q, 1), bdet)], dim=1)
            return ["rec", rec, M, max_results, c.key32(qp)]
        return ["pending", self._local_submit(qp, M, threshold), M, max_results, c.key32(qp)]

    def progressive_finish(self, p):
        """Gather and merge a submitted batch (once: the handle then holds the results)."""
        if p[0] == "done":
            return p[1]
        rec = p[1] if p[0] == "rec" else self._local_finish(p[1])
        out = self.merge(all_gather(rec, self.group, self.comm), p[2], p[3], p[4])
        p[:] = ["done", out]
        return out

    def brute_force(self, queries, max_results: int):
        """Global top-k by the overall score: local top-k, all-gather, R-way merge."""
        t = torch()
        c = self.local
        qp = c.prepare_queries(queries)
        Q = qp.N
        k = max(1, int(max_results))
        sc, ids, _, _, _ = c.exact_topk(qp, 1, k)
        det = K.rescore(qp, c.prep, ids, c.id_base)
        g = all_gather(pack(sc, ids, det), self.group, self.comm)
        gs, gi, gd = unpack(g)
        R = g.shape[0]
        none_s = t.full((R, Q), -float("inf"), dtype=t.float64, device=g.device)
        none_i = t.full((R, Q), -1, dtype=t.int64, device=g.device)
        none_d = t.zeros((R, Q, gd.shape[-1]), dtype=t.float64, device=g.device)
        # lists are sorted by overall (score desc, id asc); the final stable sort by overall keeps it
        oid, odet, cnt = K.progressive_final(gs, gi, gd, none_s, none_i, none_d, k, key32=c.key32(qp))
        return oid, odet[..., 0], odet[..., 1:], cnt

    def frame_search(self, queries, max_results: int, threshold: float = 0.1):
        """Global level-0 scan (> threshold), merged across shards."""
        t = torch()
        c = self.local
        qp = c.prepare_queries(queries)
        Q = qp.N
        k = max(1, int(max_results))
        sc, ids, _, _, _ = c.exact_topk(qp, 0, k, float(threshold), 2)
        g = all_gather(pack(sc, ids, sc.unsqueeze(-1)), self.group, self.comm)
        gs, gi, gd = unpack(g)
        R = g.shape[0]
        none_s = t.full((R, Q), -float("inf"), dtype=t.float64, device=g.device)
        none_i = t.full((R, Q), -1, dtype=t.int64, device=g.device)
        none_d = t.zeros((R, Q, 1), dtype=t.float64, device=g.device)
        oid, odet, cnt = K.progressive_final(gs, gi, gd, none_s, none_i, none_d, k, key32=c.key32(qp))
        return oid, odet[..., 0], cnt
