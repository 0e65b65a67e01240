"""Progressive similarity search on MI355X.

`ProgressiveSimilaritySearchEngine` is the drop-in for the reference's core/search_engine.py:23-388
(same constructor, methods, ordering and result objects); `IndexCorpus` is the batched device-
resident form: index vectors are prepared once (hq_seg_prepare) and a query batch is answered by the
fused MFMA scan (hq_scan_topk) + re-scoring (hq_rescore) + final ranking (hq_progressive_final).

Ordering contract (reference): candidates are ranked by score descending with Python's stable sort,
i.e. ties keep candidate-pool order — (score desc, pool index asc).  Progressive search keeps the
level-0 top `max_candidates_per_level` among sims >= threshold (first arg-max if none pass), then
stable-sorts those survivors by the overall score.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import kernels as K
from .._dev import is_tensor, to_dev, to_np, torch
from ..models import QuantizedModel, SearchResult
from .._compat import bases as _bases

MAX_FUSED_K = 64     # list length of the f64 scans (hq_scan_topk)
MAX_SPLIT_K = 1024   # list length of the split-f16 scans (k > 64: LDS-sorted pools, tiled re-rank)
_FUSED_FINAL = True  # long lists: the final ranking inside the re-rank's sort (hq_refine_final_ws); False: A/B
# How progressive_finish learns a batch's redo count: "copy" — a pinned copy queued behind the re-rank, read
# after the event behind it; "side" — an event right after the re-rank and the count read after it on a side
# stream (no copy on the search stream).  A/B, one box (profiles/r06_ab_count_read.txt): "side" measured
# 2% (M = 20) to 7% (M = 100) slower — the host's extra copy and stream sync per finish outweigh the ~4 us
# copy kernel it takes off the search stream — so "copy" stays the default.  Two forms where the re-rank
# kernel itself hands the count to pinned host memory measured slower too (profiles/r06_ab_count_kernel.txt):
# the last workgroup to finish (a ticket atomic per workgroup; M = 20 5.5M -> 5.3M QPS) and a system-scope
# store of each query's redo flag (5.5M -> 5.2M).  So did the copy queued at submit on a side stream that waits
# for the re-rank's event (5.82-5.83M -> 5.67-5.69M at three batches in flight).
_COUNT_READ = "copy"
_RING = 16  # redo counters per (device, stream, thread): a slot is re-cleared _RING - 1 batches later


@dataclass
class LevelConfig:
    grid_size: int
    start_index: int
    end_index: int
    is_offset_sampling: bool = False


def _f64(x):
    t = torch()
    return to_dev(x, t.float64)


def _idx(x):
    """Host index vector as f64, or kept f32 when it is f32 (IndexCorpus then applies the f32 statistics)."""
    a = np.asarray(x)
    return a if a.dtype == np.float32 else a.astype(np.float64, copy=False)


def _is_f32(x) -> bool:
    """float32 index vectors: the reference's np.std/np.mean then run in f32 (search_engine.py:153-159)."""
    dt = getattr(x, "dtype", None)
    if dt is None:
        return False
    return dt == np.float32 or str(dt) == "torch.float32"


def _stack_rows(rows):
    """Equal-length index vectors -> ([N, L] f64 array, per-row float32 flags or None).  Pools mixing
    float32 and float64 vectors keep each row's dtype semantics (hq_seg_prepare_rows)."""
    flags = np.array([_is_f32(r) for r in rows], dtype=bool)
    if flags.all():
        return np.stack([np.asarray(r) for r in rows]), None
    if not flags.any():
        return np.stack([np.asarray(r, dtype=np.float64) for r in rows]), None
    return np.stack([np.asarray(r, dtype=np.float64) for r in rows]), flags


# level scores the reference returns as Python floats (constant branches, clamps); any other value
# of a float32 comparison is a numpy float32 (core/search_engine.py:141-174)
_PY_LEVEL_VALUES = (0.0, 0.1, 1.0)

# Threshold typing (NumPy 2, NEP 50): the reference compares a numpy float32 level score with the
# Python-float threshold in float32 (`s >= t` is `s >= float32(t)`), a Python-float score in float64.
# The exact re-rank kernels apply that per pair (hq_search.hip typed_pass: the level score's type is known
# there); the dense exact path splits each row's candidates by score type (_select_typed).  Thresholds are
# therefore always passed as given.


def combine_levels(lv: np.ndarray, both32: bool) -> np.ndarray:
    """_calculate_overall_similarity (search_engine.py:191-230) from per-level scores [N, nl]: running
    sum of score * 1/(l+1), divide, clamp.  both32: the level scores came from float32 arrays, so a
    value outside (0, 0.1, 1) is a numpy float32 and the sum turns float32 once one enters (NEP 50)."""
    N, nl = lv.shape
    tws = np.zeros(N)
    acc32 = np.zeros(N, dtype=bool)
    tw = 0.0
    for l in range(nl):
        v, w = lv[:, l], 1.0 / (l + 1)
        t32 = (~np.isin(v, _PY_LEVEL_VALUES)) if both32 else np.zeros(N, dtype=bool)
        term = np.where(t32, (v.astype(np.float32) * np.float32(w)).astype(np.float64), v * w)
        f32sum = (tws.astype(np.float32) + term.astype(np.float32)).astype(np.float64)
        tws = np.where(acc32 | t32, f32sum, tws + term)
        acc32 = acc32 | t32
        tw += w
    out = np.where(acc32, (tws.astype(np.float32) / np.float32(tw)).astype(np.float64), tws / tw if tw > 0 else 0.0)
    return np.maximum(0.0, np.minimum(1.0, out))


_REDO_WARM = False  # IndexCorpus._warm_redo ran in this process
_WARM_LOCK = threading.Lock()


def _lock(obj):
    """The object's lock (created on first use; dict.setdefault is atomic under the GIL)."""
    lk = obj.__dict__.get("_lock_")
    return lk if lk is not None else obj.__dict__.setdefault("_lock_", threading.RLock())


class PendingSearch:
    """A progressive search batch queued on the GPU (IndexCorpus.progressive_submit): its device outputs,
    the pinned copy of its redo count and the event behind that copy; `done` holds the results of the
    synchronous paths (small corpora, dense exact path)."""

    __slots__ = ("done", "qp", "out", "res", "cnt", "forced", "nredo", "event", "threshold", "M", "K_out", "kp",
                 "ring")

    def __init__(self, done=None, qp=None, out=None, res=None, cnt=None, forced=None, nredo=None, event=None,
                 threshold=0.0, M=0, K_out=0, kp=0, ring=None):
        self.done, self.qp, self.out, self.res, self.cnt, self.forced = done, qp, out, res, cnt, forced
        self.nredo, self.event, self.threshold, self.M, self.K_out = nredo, event, threshold, M, K_out
        self.kp = kp  # the first pass's list length (the retry's base)
        self.ring = ring  # side reads: (ring entry, slot) of the batch's device counter


class IndexCorpus:
    """A corpus of equal-length hierarchical index vectors resident in HBM.

    `indices`: [N, L] (NumPy or device tensor); `id_base`: global id of row 0 (corpus shards).

    Every ranking is EXACT: the fused MFMA scan (approximate scores, |err| << EPS) produces a list
    of SLACK extra candidates per query, hq_refine_topk re-scores the list in the reference's
    operation order and proves (or not) that nothing outside the list can enter the exact top-k;
    unproven queries and the "none passed" fallback are answered by the dense exact path.

    Re-entrant: the reference calls its engines from ThreadPoolExecutor workers (core/video_search.py:806,
    854; core/streaming_processor.py:294), so one corpus may serve many threads at once.  Every piece of
    per-call device state (scan / re-rank workspace, redo counters) is keyed by thread as well as stream,
    and the host-side caches (pinned buffers, statistics, adaptive list lengths) are guarded by a lock."""

    # bound on |approximate - exact| score: the level-0 scan contracts in split f16 on the matrix cores
    # (|dscore| <= ~5.5e-6, hq_mi355x.h), the other scans in f64 (< 1e-13)
    EPS = 2e-5
    SLACK = 8

    def __init__(self, indices, id_base: int = 0, row_f32=None):
        f32 = _is_f32(indices)
        x = _f64(indices)
        if x.dim() != 2:
            raise ValueError("IndexCorpus expects a 2-D [N, L] array of index vectors")
        self.N, self.L = int(x.shape[0]), int(x.shape[1])
        self.id_base = int(id_base)
        self.prep = K.flag_rows(K.packov(K.pack0(K.seg_prepare(x, src_f32=f32, row_f32=None if f32 else row_f32))))
        self.nseg = self.prep.nseg
        # float32 rows outside the scans' model (values whose squares under/overflow in float32): the
        # whole corpus then takes the dense exact path (one host sync, at build time, f32 corpora only)
        self.dense_only = bool(self.prep.unsafe_rows().any()) if self.prep.f32 and self.N else False
        # the prepared layouts are written on the building thread's stream: a search on another stream waits
        # for them (an event wait queued on the device, no host sync)
        self._built_on = K.stream()
        self._ready = torch().cuda.Event()
        self._ready.record()
        self._warm_redo(x)

    def _warm_redo(self, x):
        """Once per process, with the first corpus built: one 1-query progressive batch whose list is marked
        unproven, so the redo path (the longer-list retry, its re-rank, the torch selections and scatters
        around them) runs once at build time.  ROCm loads a kernel's code object on its first launch (several
        ms per torch kernel), and without this the first batch that needs a redo paid that for a dozen kernels:
        57 ms against 1.2 ms warm for the clustered corpus's first batch (profiles/r06_cold_batch.txt)."""
        global _REDO_WARM
        M = 20  # HilbertQuantizer's max_candidates_per_level
        with _WARM_LOCK:
            if _REDO_WARM or self.N <= M or M + self.SLACK > self._max_list(0) or self.dense_only \
                    or not self._fused_ok(0) or self._retry_len(0, M + self.SLACK) is None:
                return
            _REDO_WARM = True
        p = self.progressive_submit(x[:1], 10, 0.1, M)
        if p.done is None and p.ring is None:
            p.event.synchronize()
            p.res.zero_()           # the batch's one list "unproven": the retry path runs
            p.nredo[0] = 1
            self.progressive_finish(p)
        self.reset_stats()

    def prepare_queries(self, queries, row_f32=None) -> "K.Prepared":
        """queries: [Q, L] (or [L]); a pair (array, per-row float32 flags) for mixed-dtype batches."""
        if isinstance(queries, tuple):
            queries, row_f32 = queries
        if K.stream() != self._built_on:
            torch().cuda.current_stream().wait_event(self._ready)
        f32 = _is_f32(queries)
        q = _f64(queries)
        if q.dim() == 1:
            q = q.view(1, -1)
        if q.shape[1] != self.L:
            raise ValueError(f"query index length {q.shape[1]} != corpus index length {self.L}")
        # the overall (brute-force) layout is attached by the first overall scan of the batch (scan_topk)
        return K.seg_prepare_pack0(q, src_f32=f32, row_f32=None if f32 else row_f32)

    def _fused_ok(self, mode: int) -> bool:
        """The fused scans hold the contracted columns in registers: <= 256 padded values (hq_scan_topk)."""
        if mode == 0:
            return K.seg_level0_len(self.L) <= 256
        return self.prep.Lp <= 256

    def _max_list(self, mode: int) -> int:
        """Longest scan list (k + SLACK) the scan for `mode` takes: the split-f16 scans (level-0 copies for
        mode 0, the overall layout for mode 1) up to MAX_SPLIT_K, the f64 scans up to MAX_FUSED_K."""
        if self.L % 2 or K._lib.get_option("scan_v1") is not None:
            return MAX_FUSED_K
        if (mode == 0 and self.prep.Z16 is not None) or (mode == 1 and self.prep.Zov16 is not None):
            return MAX_SPLIT_K
        return MAX_FUSED_K

    def key32(self, qp) -> bool:
        """Every vector float32 (query batch and corpus): the reference's sorts then compare numpy float32
        and Python-float scores in float32 (NEP 50), so rankings use float32-rounded keys (K.THR_KEY32)."""
        return bool(self.prep.all32 and qp.all32)

    def _forced(self, qp):
        """Device bool [Q] of queries that must take the dense exact path (float32 outside the model)."""
        t = torch()
        if self.dense_only:
            return t.ones(qp.N, dtype=t.bool, device=qp.Z.device)
        return qp.unsafe_rows() if qp.f32 else None

    # ---- scores ------------------------------------------------------------------------------
    def level_scores(self, queries, level: int):
        """Dense exact [Q, N]: level >= 0 -> compare_indices_at_level, -1 -> overall similarity."""
        return K.level_scores(self.prepare_queries(queries), self.prep, level)

    def _dense(self, qp, sel, mode: int, k: int, thr: float, thr_mode: int):
        """Dense exact path for the queries `sel` (device int64): scores, select top-k + arg-max."""
        sub = qp.rows(sel)
        outs = []
        chunk = max(1, (1 << 27) // max(1, self.N))  # <= 1 GiB of scores per launch
        typed = (mode == 0 and thr_mode != 0 and float(np.float32(thr)) != float(thr) and sub.f32 and self.prep.f32)
        key32 = self.key32(sub)
        for i in range(0, sub.N, chunk):
            part = sub.rows(torch().arange(i, min(sub.N, i + chunk), device=sel.device))
            sc = K.level_scores(part, self.prep, 0 if mode == 0 else -1)
            if key32:
                outs.append(self._select_key32(sc, k, float(thr), thr_mode))
            elif typed:
                outs.append(self._select_typed(part, sc, k, float(thr), thr_mode))
            else:
                outs.append(K.select_topk(sc, k, thr, thr_mode, self.id_base))
        return [torch().cat([o[j] for o in outs], 0) for j in range(4)]

    def _select_typed(self, qp, sc, k: int, thr: float, thr_mode: int):
        """select_topk of level scores where float32(thr) != thr and float32 vectors are involved: the
        numpy-float32 scores (both vectors float32, general branch: a value outside 0 / 0.1 / 1) are tested
        against float32(thr), the Python-float ones against thr (NEP 50).  The top-k of each kind (the other
        kind masked to -inf) merge by (score desc, id asc) into the row's top-k; the first arg-max is the
        better of the two."""
        t = torch()
        qf = (qp.S[:, 0, 3].to(t.int64) & 1).bool()
        cf = (self.prep.S[:, 0, 3].to(t.int64) & 1).bool()
        py = (sc == 0.0) | (sc == 0.1) | (sc == 1.0)
        f32 = qf.view(-1, 1) & cf.view(1, -1) & ~py
        ninf = t.tensor(-float("inf"), dtype=sc.dtype, device=sc.device)
        sa, ia, ba, bia = K.select_topk(t.where(f32, sc, ninf), k, float(np.float32(thr)), thr_mode, self.id_base)
        sb, ib, bb, bib = K.select_topk(t.where(f32, ninf, sc), k, thr, thr_mode, self.id_base)
        s, i = t.cat([sa, sb], 1), t.cat([ia, ib], 1)
        key = t.where(i >= 0, i, t.full_like(i, 2 ** 62))
        o = t.argsort(key, dim=1, stable=True)
        s, i = s.gather(1, o), i.gather(1, o)
        o = t.argsort(s, dim=1, descending=True, stable=True)[:, :k]
        s, i = s.gather(1, o), i.gather(1, o)
        i = t.where(s > -float("inf"), i, t.full_like(i, -1))
        pick_b = (bb > ba) | ((bb == ba) & (bib < bia))
        return s, i, t.where(pick_b, bb, ba), t.where(pick_b, bib, bia)

    def _select_key32(self, sc, k: int, thr: float, thr_mode: int):
        """select_topk for all-float32 searches: the threshold test typed per value (a numpy float32 score
        against float32(thr), a Python-float one - 0, 0.1, 1 - against thr), the order by float32-rounded
        keys (score desc, id asc), the first arg-max by key; the scores returned are the exact values."""
        t = torch()
        sk = sc.to(t.float32).to(t.float64)
        ninf = t.full_like(sk, -float("inf"))
        ok = None
        if thr_mode:
            py = (sc == 0.0) | (sc == 0.1) | (sc == 1.0)
            tt = t.where(py, t.full_like(sc, thr), t.full_like(sc, float(np.float32(thr))))
            ok = (sc >= tt) if thr_mode == 1 else (sc > tt)
        _, oi, _, _ = K.select_topk(sk if ok is None else t.where(ok, sk, ninf), k, 0.0, 0, 0)
        valid = oi >= 0
        if ok is not None:
            valid = valid & ok.gather(1, oi.clamp(min=0))
        os_ = t.where(valid, sc.gather(1, oi.clamp(min=0)), t.full_like(oi, 0, dtype=sc.dtype) - float("inf"))
        oi = t.where(valid, oi + self.id_base, t.full_like(oi, -1))
        bi = t.argmax(sk, dim=1)  # the first maximal key
        return os_, oi, sc.gather(1, bi.view(-1, 1)).view(-1), bi + self.id_base

    def exact_topk(self, qp, mode: int, k: int, thr: float = 0.0, thr_mode: int = 0, need_best: bool = False):
        """Exact per-query top-k (score desc, id asc) among candidates passing the threshold test;
        with need_best, also the exact first arg-max for queries where nothing passed.
        Returns (scores [Q, k], ids [Q, k], count [Q], best [Q], best_id [Q])."""
        t = torch()
        Q = qp.N
        dev = qp.Z.device
        best = t.full((Q,), -float("inf"), dtype=t.float64, device=dev)
        bid = t.full((Q,), -1, dtype=t.int64, device=dev)
        kp = k + self.SLACK
        if kp > self._max_list(mode) or self.dense_only or not self._fused_ok(mode):
            sc, ids, b, bi = self._dense(qp, t.arange(Q, device=dev), mode, k, thr, thr_mode)
            cnt = (ids >= 0).sum(1).to(t.int32)
            return sc, ids, cnt, b, bi
        lo_mode = 0 if thr_mode == 0 else 1
        asc, aid, _, _ = K.scan_topk(qp, self.prep, mode, kp, thr - self.EPS, lo_mode, self.id_base)
        tm = thr_mode | (K.THR_KEY32 if self.key32(qp) else 0)
        sc, ids, cnt, res = K.refine_topk(qp, self.prep, mode, asc, aid, k, thr, tm, self.EPS, self.id_base)
        redo = (res == 0)
        if need_best:
            redo = redo | (cnt == 0)
        forced = self._forced(qp)
        if forced is not None:
            redo = redo | forced
        sel = t.nonzero(redo).view(-1)
        if sel.numel():
            # unproven lists (near-ties at the list end, short lists) first get the scan path with a longer
            # list; nothing-passed rows (arg-max), forced rows and what stays unproven take the dense path
            try_ = res[sel] == 0
            if need_best:
                try_ = try_ & (cnt[sel] > 0)
            if forced is not None:
                try_ = try_ & ~forced[sel]
            rsel = sel[try_]
            if rsel.numel():
                got = self._retry_scan(qp.rows(rsel), mode, k, thr, thr_mode, kp, det=False)
                if got is not None:
                    s2, i2, c2, r2 = got
                    ok = (r2 == 1) & (c2 > 0) if need_best else (r2 == 1)
                    sc[rsel[ok]], ids[rsel[ok]], cnt[rsel[ok]] = s2[ok], i2[ok], c2[ok]
                    keep = t.ones(sel.numel(), dtype=t.bool, device=dev)
                    keep[t.nonzero(try_).view(-1)[ok]] = False
                    sel = sel[keep]
        if sel.numel():
            self._bump(dense_queries=int(sel.numel()))
            s2, i2, b2, bi2 = self._dense(qp, sel, mode, k, thr, thr_mode)
            sc[sel] = s2
            ids[sel] = i2
            cnt[sel] = (i2 >= 0).sum(1).to(t.int32)
            best[sel] = b2
            bid[sel] = bi2
        return sc, ids, cnt, best, bid

    RETRY_FACTOR = 4
    _count_read = _COUNT_READ
    ADAPT_LISTS = True  # a batch that mostly needed the retry lengthens later first passes at its M (slack_for)

    def _retry_len(self, mode: int, cur: int):
        """List length of the longer-list retry after a first pass of `cur` entries, or None when no retry
        pays: the f64 scans (option scan_v1, odd L) keep the dense path (their lists stop at 64 and their LDS
        tiles grow with the list), and a retry that would not at least double the list (M = 1000: 1008 ->
        1024) is a full re-scan for a few entries, so those rows go straight to the dense path."""
        kp2 = min(self._max_list(mode), self.RETRY_FACTOR * cur)
        if kp2 < 2 * cur or self._max_list(mode) <= MAX_FUSED_K or not self._fused_ok(mode) or self.dense_only:
            return None
        return kp2

    def _retry_scan(self, qp, mode: int, k: int, thr: float, thr_mode: int, cur: int, det: bool = False):
        """The scan path again for queries whose list was not proven complete, with a list RETRY_FACTOR
        times longer than the first pass's `cur` entries (at most the scan's limit): a list ends in near-ties
        when more than its slack of candidates lie within EPS of the k-th (runs of near-duplicates in the
        corpus), or short when the sampled starting threshold overshot.  None when no longer list pays
        (_retry_len).  Returns refine_topk's (scores, ids, count, resolved) (+ det, the [overall, levels]
        records, with det)."""
        kp2 = self._retry_len(mode, cur)
        if kp2 is None:
            return None
        self._bump(retry_queries=qp.N)
        lo_mode = 0 if thr_mode == 0 else 1
        asc, aid, _, _ = K.scan_topk(qp, self.prep, mode, kp2, thr - self.EPS, lo_mode, self.id_base)
        tm = thr_mode | (K.THR_KEY32 if self.key32(qp) else 0)
        if det:
            return K.refine_rescore_topk(qp, self.prep, mode, asc, aid, k, thr, tm, self.EPS, self.id_base,
                                         count_empty=True)
        return K.refine_topk(qp, self.prep, mode, asc, aid, k, thr, tm, self.EPS, self.id_base, count_empty=True)

    def _level0_redo(self, qp, sel, M: int, thr: float, res, cnt, forced, kp: int = 0):
        """Exact level-0 top-M (>= thr) records of the queries `sel` the first pass left unproven or empty:
        unproven lists where something passed are re-scanned with a longer list (_retry_scan); the rest —
        nothing passed (the arg-max fallback), forced rows, lists the retry leaves unproven — take the dense
        exact path.  kp: the first pass's list length (default M + SLACK).
        Returns (s0 [n, M], ids [n, M], best [n], bid [n], det [n, M, W], bdet [n, W])."""
        t = torch()
        n, dev, W = int(sel.numel()), sel.device, 1 + self.nseg
        s0 = t.full((n, M), -float("inf"), dtype=t.float64, device=dev)
        ids = t.full((n, M), -1, dtype=t.int64, device=dev)
        best = t.full((n,), -float("inf"), dtype=t.float64, device=dev)
        bid = t.full((n,), -1, dtype=t.int64, device=dev)
        det = t.zeros((n, M, W), dtype=t.float64, device=dev)
        bdet = t.zeros((n, W), dtype=t.float64, device=dev)
        need = t.ones(n, dtype=t.bool, device=dev)
        try_ = (res[sel] == 0) & (cnt[sel] > 0)
        if forced is not None:
            try_ = try_ & ~forced[sel]
        r = t.nonzero(try_).view(-1)
        cur = int(kp) if kp else M + self.SLACK
        if r.numel():
            got = self._retry_scan(qp.rows(sel[r]), 0, M, thr, 1, cur, det=True)
            if got is not None:
                s2, i2, c2, r2, d2 = got
                ok = (r2 == 1) & (c2 > 0)
                rr = r[ok]
                s0[rr], ids[rr], det[rr] = s2[ok], i2[ok], d2[ok]
                need[rr] = False
                if (self.ADAPT_LISTS and r.numel() >= max(8, qp.N // 10) and cur == M + self.SLACK
                        and rr.numel() * 2 >= r.numel()):
                    # a tenth of the batch or more ended in near-ties (runs of near-duplicates in the corpus) and
                    # the longer list resolved most of them: later batches at this M take the retry's list
                    # length on the first pass (one scan instead of a scan plus a retry per batch; results are
                    # exact either way).  Only when a retry ran: the scans without one keep their length.
                    with _lock(self):
                        self.__dict__.setdefault("_slack", {})[int(M)] = self._retry_len(0, cur) - M
        d = t.nonzero(need).view(-1)
        if d.numel():
            self._bump(dense_queries=int(d.numel()))
            dsel = sel[d]
            sub = qp.rows(dsel)
            s3, i3, b3, bi3 = self._dense(qp, dsel, 0, M, thr, 1)
            s0[d], ids[d], best[d], bid[d] = s3, i3, b3, bi3
            det[d] = K.rescore(sub, self.prep, i3, self.id_base)
            bdet[d] = K.rescore(sub, self.prep, bi3.view(-1, 1), self.id_base).view(-1, W)
        return s0, ids, best, bid, det, bdet

    # ---- searches ----------------------------------------------------------------------------
    def brute_force(self, queries, max_results: int):
        """search_engine.py:302-338 for a query batch -> (ids [Q, K], overall [Q, K], levels [Q, K, nseg])."""
        qp = self.prepare_queries(queries)
        k = max(1, min(int(max_results), self.N)) if self.N else 1
        _, ids, _, _, _ = self.exact_topk(qp, 1, k)
        det = K.rescore(qp, self.prep, ids, self.id_base)
        return ids, det[..., 0], det[..., 1:]

    def progressive(self, queries, max_results: int, threshold: float = 0.1, max_candidates_per_level: int = 100):
        """search_engine.py:232-300 + :340-388 for a query batch.
        Returns (ids [Q, K], overall [Q, K], levels [Q, K, nseg], count [Q]) with K = max_results;
        rows are padded with id -1 beyond count."""
        return self.progressive_finish(self.progressive_submit(queries, max_results, threshold,
                                                               max_candidates_per_level))

    def progressive_submit(self, queries, max_results: int, threshold: float = 0.1,
                           max_candidates_per_level: int = 100) -> "PendingSearch":
        """Queue a progressive search without waiting for it: the scan, exact re-rank, re-score and final
        ranking are launched on the current stream and the count of queries needing the dense exact path
        is copied to pinned host memory behind them.  `progressive_finish` waits for that copy alone, so
        batch i + 1 can be queued before batch i is finished (the GPU never idles on the host)."""
        t = torch()
        qp = self.prepare_queries(queries)
        Q = qp.N
        K_out = max(1, int(max_results))
        M = int(max_candidates_per_level)
        if self.N <= M:
            # the level loop never filters (:298): every candidate is re-scored and stable-sorted
            ids, ov, lv = self.brute_force(queries, min(K_out, max(self.N, 1)))
            cnt = (ids >= 0).sum(dim=1).to(t.int32)
            return PendingSearch(done=(ids, ov, lv, cnt))
        if M + self.SLACK > self._max_list(0) or self.dense_only or not self._fused_ok(0):
            s0, ids, cnt, best, bid = self.exact_topk(qp, 0, M, float(threshold), 1, need_best=True)
            oid, odet, ocnt = self._final(qp, s0, ids, best, bid, K_out)
            return PendingSearch(done=(oid, odet[..., 0], odet[..., 1:], ocnt))
        nredo, nnext, ring = self._redo_counter(qp.Z.device, self._count_read == "side")
        # queries forced onto the dense path (float32 outside the scans' model) join the redo count on the
        # device, so finishing still waits for one value only
        forced = self._forced(qp)
        kp = M + self.slack_for(M)
        cnt, res, oid, odet, ocnt = self._scan_refine_final(qp, M, float(threshold), nredo, nnext, K_out, kp)
        if forced is not None:
            nredo.add_(forced.sum(dtype=t.int32).view(1))
        if ring is not None:
            # the slot stays untouched until _RING - 1 batches later (and is read before that: _redo_counter);
            # finish reads it after this event
            ev = t.cuda.Event()
            ev.record()
            p = PendingSearch(qp=qp, out=(oid, odet, ocnt), res=res, cnt=cnt, forced=forced, nredo=nredo,
                              event=ev, threshold=float(threshold), M=M, K_out=K_out, kp=kp, ring=ring)
            with _lock(self):
                ring[0][2][ring[1]] = p
            return p
        # the counter's value leaves now, behind the re-rank (a last-workgroup write of it to the pinned int from
        # the re-rank kernel measured slower: 21 -> 43 us, every workgroup's release fence)
        host = self._pinned(nredo.dtype)
        host.copy_(nredo, non_blocking=True)
        ev = t.cuda.Event()
        ev.record()
        return PendingSearch(qp=qp, out=(oid, odet, ocnt), res=res, cnt=cnt, forced=forced,
                             nredo=host, event=ev, threshold=float(threshold), M=M, K_out=K_out, kp=kp)

    def progressive_finish(self, p: "PendingSearch"):
        """Wait for a submitted batch's redo count (the one host sync) and recompute the queries whose
        list is not proven complete or where nothing passed, by the dense exact path."""
        if p.done is not None:
            return p.done
        t = torch()
        oid, odet, ocnt = p.out
        if p.ring is not None:
            nredo = self._resolve(p)
        else:
            p.event.synchronize()
            nredo = int(p.nredo[0])
            self._unpin(p.nredo)  # read: reusable
        self._bump(batches=1, queries=p.qp.N)
        if nredo > 0:
            # the redo's time on the stream, between two events read lazily (stats): no host sync here, so the
            # host goes on queueing batches while the redo runs
            e0 = t.cuda.Event(enable_timing=True)
            e0.record()
            redo = (p.res == 0) | (p.cnt == 0)
            if p.forced is not None:
                redo = redo | p.forced
            sel = t.nonzero(redo).view(-1)
            n = int(sel.numel())
            if n:
                s2, i2, b2, bi2, d2, bd2 = self._level0_redo(p.qp, sel, p.M, p.threshold, p.res, p.cnt, p.forced,
                                                             kp=p.kp)
                o2, dd2, c2 = self._final(p.qp.rows(sel), s2, i2, b2, bi2, p.K_out, bdet=bd2, det=d2)
                oid[sel], odet[sel], ocnt[sel] = o2, dd2, c2
            e1 = t.cuda.Event(enable_timing=True)
            e1.record()
            self._bump(redo_batches=1, redo_queries=n, _events=(e0, e1))
        p.done = (oid, odet[..., 0], odet[..., 1:], ocnt)  # finishing again returns the same results
        return p.done

    _STAT_KEYS = ("batches", "queries", "redo_batches", "redo_queries", "retry_queries", "dense_queries")

    @property
    def stats(self) -> dict:
        """Counters of the submitted progressive batches: batches / queries finished, batches and queries
        redone after the first pass (short or unproven lists, nothing passing, forced rows), and the
        stream time spent there (dense_s: between two events around each redo, read here — this waits for
        the redos still running); of the redone queries, those re-scanned with a longer list (retry_queries)
        and those scored densely (dense_queries).  A snapshot: later batches do not change it."""
        with _lock(self):
            st = self.__dict__.setdefault("_stats", dict.fromkeys(self._STAT_KEYS, 0))
            evs = self.__dict__.setdefault("_stat_events", [])
            done, evs[:] = list(evs), []
            st["dense_s"] = st.get("dense_s", 0.0)
        dt = 0.0
        for e0, e1 in done:
            e1.synchronize()
            dt += e0.elapsed_time(e1) / 1e3
        with _lock(self):
            st["dense_s"] += dt
            return dict(st)

    def _bump(self, _events=None, **counts):
        with _lock(self):
            st = self.__dict__.setdefault("_stats", dict.fromkeys(self._STAT_KEYS, 0))
            for key, v in counts.items():
                st[key] += v
            if _events is not None:
                self.__dict__.setdefault("_stat_events", []).append(_events)

    def reset_stats(self):
        with _lock(self):
            self.__dict__.pop("_stats", None)
            self.__dict__.pop("_stat_events", None)

    def _pinned(self, dtype):
        """A one-element pinned host buffer: recycled once its batch is finished (a fresh pinned
        allocation per batch can stall the host between launches)."""
        with _lock(self):
            free = self.__dict__.setdefault("_pinned_free", {}).setdefault(dtype, [])
            if free:
                return free.pop()
        return torch().empty(1, dtype=dtype, pin_memory=True)

    def _unpin(self, buf):
        """Return a pinned buffer whose value has been read."""
        with _lock(self):
            self.__dict__.setdefault("_pinned_free", {}).setdefault(buf.dtype, []).append(buf)

    def _redo_counter(self, dev, side: bool = False):
        """(counter, next, ring): device int32 [1] views of a ring of _RING counters used in turn by ONE thread
        on one stream — the exact re-rank counts this batch's queries needing the dense path in `counter`
        (zero on entry) and clears `next`, the following batch's counter (hq_refine_rescore_topk_pp: no memset
        launch per batch), so a slot is cleared again _RING - 1 batches later; ring[2] counts the batches whose
        slot is still to be read (progressive_finish).  Keyed by thread too: two threads sharing a stream would
        otherwise take slots of one ring and clear each other's count before it is read."""
        t = torch()
        key = (str(dev), K.stream(), threading.get_ident())
        with _lock(self):
            cache = self.__dict__.setdefault("_redo", {})
            ent = cache.get(key)
            if ent is None:
                ent = cache[key] = [t.zeros(_RING, dtype=t.int32, device=dev), 0, [None] * _RING]
            buf, i = ent[0], ent[1]
            ent[1] = (i + 1) % _RING
            j = (i + 1) % _RING
            old = ent[2][j]  # a batch still unread whose slot this batch's re-rank clears: read it first
        if old is not None:
            self._resolve(old)
        return buf[i:i + 1], buf[j:j + 1], ((ent, i) if side else None)

    def _resolve(self, p) -> int:
        """A side-read batch's redo count (once): wait for its event, read its slot, free the slot."""
        with _lock(self):
            if isinstance(p.nredo, int):
                return p.nredo
        p.event.synchronize()
        v = self._side_read(p.nredo)
        with _lock(self):
            if not isinstance(p.nredo, int):
                ent, i = p.ring
                if ent[2][i] is p:
                    ent[2][i] = None
                p.nredo = v
        return v

    def _side_read(self, slot) -> int:
        """The value of a finished batch's device counter, read on this thread's side stream (the search
        stream goes on with the next batch's kernels; no copy is queued on it)."""
        t = torch()
        key = (slot.device.index, threading.get_ident())
        with _lock(self):
            ss = self.__dict__.setdefault("_side", {})
            st = ss.get(key)
            if st is None:
                st = ss[key] = (t.cuda.Stream(device=slot.device), t.empty(1, dtype=slot.dtype, pin_memory=True))
        side, host = st
        with t.cuda.stream(side):
            host.copy_(slot, non_blocking=True)
        side.synchronize()
        return int(host[0])

    def _no_fallback(self, Q: int, dev):
        """Constant (-inf, -1, zeros) fallback slot of a batch of Q queries, cached per stream: the fills
        are stream-ordered, so a batch on another stream must not read them before they ran."""
        t = torch()
        cache = self.__dict__.setdefault("_nofb", {})
        key = (Q, str(dev), K.stream())
        if key not in cache:
            cache[key] = (t.full((Q,), -float("inf"), dtype=t.float64, device=dev),
                          t.full((Q,), -1, dtype=t.int64, device=dev),
                          t.zeros((Q, 1 + self.nseg), dtype=t.float64, device=dev))
        return cache[key]

    def reset_list_lengths(self):
        """Forget the first-pass list lengths the corpus adapted (slack_for): back to SLACK at every M."""
        with _lock(self):
            self.__dict__.pop("_slack", None)

    def slack_for(self, M: int) -> int:
        """Extra list entries of the first pass at list length M: SLACK, or the longer list a corpus with
        runs of near-duplicates showed it needs (_level0_redo: most lists of a batch ended in near-ties)."""
        with _lock(self):
            return self.__dict__.get("_slack", {}).get(int(M), self.SLACK)

    def _scan_refine(self, qp, mode: int, k: int, thr: float, thr_mode: int, nredo=None, det: bool = False,
                     next_redo=None, slack=None):
        """Fused scan (slack, default SLACK, extra list entries) + exact re-rank; resolved[q] == 0 marks an
        unproven list.  nredo: device counter of queries needing the dense path (unresolved or nothing
        passed).  det: also the exact [overall, levels] re-score of the output (rows staged once)."""
        lo_mode = 0 if thr_mode == 0 else 1
        kp = k + (self.SLACK if slack is None else int(slack))
        asc, aid, _, _ = K.scan_topk(qp, self.prep, mode, kp, thr - self.EPS, lo_mode, self.id_base)
        tm = thr_mode | (K.THR_KEY32 if self.key32(qp) else 0)
        if det:
            return K.refine_rescore_topk(qp, self.prep, mode, asc, aid, k, thr, tm, self.EPS, self.id_base, redo=nredo,
                                         count_empty=True, next_redo=next_redo)
        return K.refine_topk(qp, self.prep, mode, asc, aid, k, thr, tm, self.EPS, self.id_base, redo=nredo,
                             count_empty=True)

    def _scan_refine_final(self, qp, M: int, thr: float, nredo, next_redo, K_out: int, kp: int):
        """The progressive search's first pass: level-0 scan, exact re-rank, overall re-score and final
        ranking -> (count, resolved, out_id, out_det, out_count).  On the lane-cooperative paths the re-rank's
        ranking and the final ranking are one kernel (hq_refine_final_ws: the level-0 records stay on the
        device).  No arg-max
        on this path: a query where nothing passed (count 0) is recomputed by the dense path in
        progressive_finish, so the fallback slot is a constant (-inf, id -1, zero re-scores).  kp: the list
        length (M + slack_for(M), read once by the caller)."""
        asc, aid, _, _ = K.scan_topk(qp, self.prep, 0, kp, thr - self.EPS, 1, self.id_base)
        tm = 1 | (K.THR_KEY32 if self.key32(qp) else 0)
        if _FUSED_FINAL:
            r = K.refine_final_ws(qp, self.prep, asc, aid, M, thr, tm, self.EPS, self.id_base, K_out, redo=nredo,
                                  next_redo=next_redo)
            if r is not None:
                return r
        s0, ids, cnt, res, det = K.refine_rescore_topk(qp, self.prep, 0, asc, aid, M, thr, tm, self.EPS, self.id_base,
                                                       redo=nredo, count_empty=True, next_redo=next_redo)
        best, bid, bdet = self._no_fallback(qp.N, qp.Z.device)
        oid, odet, ocnt = self._final(qp, s0, ids, best, bid, K_out, bdet, det)
        return cnt, res, oid, odet, ocnt

    def _final(self, qp, s0, ids, best, bid, K_out: int, bdet=None, det=None):
        """Exact overall + per-level re-score of the survivors and of the arg-max, then the final ranking."""
        Q = qp.N
        if det is None:
            det = K.rescore(qp, self.prep, ids, self.id_base)
        if bdet is None:
            bdet = K.rescore(qp, self.prep, bid.view(Q, 1), self.id_base).view(Q, -1)
        return K.progressive_final(s0.unsqueeze(0), ids.unsqueeze(0), det.unsqueeze(0),
                                   best.unsqueeze(0), bid.unsqueeze(0), bdet.unsqueeze(0), K_out,
                                   key32=self.key32(qp))

    def frame_search(self, queries, max_results: int, threshold: float = 0.1):
        """core/video_search.py:215-264: level-0 sim > threshold (strict), stable sort, top-k."""
        qp = self.prepare_queries(queries)
        sc, ids, _, _, _ = self.exact_topk(qp, 0, max(1, int(max_results)), float(threshold), 2)
        return ids, sc


class ProgressiveSimilaritySearchEngine(*_bases("interfaces", "SimilaritySearchEngine")):
    """Drop-in for core/search_engine.py:23 (interfaces.py:191-225 SimilaritySearchEngine)."""

    def __init__(self, similarity_threshold: float = 0.1, max_candidates_per_level: int = 100):
        self.similarity_threshold = similarity_threshold
        self.max_candidates_per_level = max_candidates_per_level
        self._pool_cache = None  # (index arrays of the last uniform pool, their resident IndexCorpus)

    # ---- structure -----------------------------------------------------------------------------
    def _parse_index_structure(self, indices, total_space: int) -> List[LevelConfig]:
        if len(indices) == 0 or total_space <= 0:
            return []
        levels = [LevelConfig(g, s, e, off) for (g, s, e, off) in K.parse_structure(int(total_space))]
        # the reference stops consuming at len(indices) (:115, :142-147); callers pass len(indices)
        return [lv for lv in levels if lv.start_index < len(indices)]

    # ---- pair scores ---------------------------------------------------------------------------
    def _corpus(self, rows) -> IndexCorpus:
        C, flags = _stack_rows(rows)
        return IndexCorpus(C, row_f32=flags)

    def _pool_corpus(self, pool) -> IndexCorpus:
        """The resident corpus of a candidate pool, re-used while the pool holds the same index arrays
        in the same order (the reference re-scores every candidate per call; re-uploading and
        re-preparing the pool per query was O(pool) host and PCIe work).  The arrays are kept
        referenced, so an identity match is a match; a QuantizedModel's hierarchical_indices are never
        written after creation (the reference's pipeline builds a new array per model)."""
        arrays = [c.hierarchical_indices for c in pool]
        with _lock(self):  # threads searching one pool share one resident corpus (built once)
            hit = self._pool_cache
            if hit is not None and len(hit[0]) == len(arrays) and all(a is b for a, b in zip(hit[0], arrays)):
                return hit[1]
            corpus = self._corpus(arrays)
            self._pool_cache = (arrays, corpus)
            return corpus

    def _scores_at_level(self, q: np.ndarray, cands: Sequence[np.ndarray], level: int) -> np.ndarray:
        """compare_indices_at_level(q, c, level) for every candidate, on the GPU."""
        N = len(cands)
        out = np.zeros(N)
        if len(q) == 0 or N == 0:
            return out
        ql = self._parse_index_structure(q, len(q))
        if level >= len(ql):
            return out
        groups: Dict[Tuple[int, bool], List[int]] = {}
        for i, c in enumerate(cands):
            groups.setdefault((len(c), _is_f32(c)), []).append(i)
        for (Lc, c32), members in groups.items():
            if Lc == 0:
                continue
            C = np.stack([_idx(cands[i]) for i in members])
            if Lc == len(q):
                corpus = IndexCorpus(C)
                s = to_np(corpus.level_scores(_idx(q)[None], level))[0]
            else:
                cl = self._parse_index_structure(C[0], Lc)
                if level >= len(cl):
                    continue
                qs, qe = ql[level].start_index, ql[level].end_index
                cs, ce = cl[level].start_index, cl[level].end_index
                m = min(qe - qs, ce - cs)
                if m <= 0:
                    continue
                qseg = _idx(q)[qs:qs + m]
                s = to_np(K.pair_scores_raw(_f64(qseg), _f64(np.ascontiguousarray(C[:, cs:cs + m])),
                                            q_f32=_is_f32(q), c_f32=c32))
            out[members] = s
        return out

    def compare_indices_at_level(self, query_indices, candidate_indices, level: int) -> float:
        if len(query_indices) == 0 or len(candidate_indices) == 0:
            return 0.0
        return float(self._scores_at_level(np.asarray(query_indices), [np.asarray(candidate_indices)], level)[0])

    def _calculate_overall_similarity(self, query_indices, candidate_indices) -> Tuple[float, Dict[int, float]]:
        ov, lv = self._overall_many(np.asarray(query_indices), [np.asarray(candidate_indices)])
        if lv.shape[1] == 0:
            return 0.0, {}
        return float(ov[0]), {i: float(lv[0, i]) for i in range(lv.shape[1])}

    def _overall_many(self, q: np.ndarray, cands: Sequence[np.ndarray]):
        ql = self._parse_index_structure(q, len(q))
        N = len(cands)
        if not ql:
            return np.zeros(N), np.zeros((N, 0))
        if all(len(c) == len(q) for c in cands) and N:
            corpus = self._corpus(cands)
            qp = corpus.prepare_queries(_idx(q)[None])
            ids = torch().arange(N, device=qp.Z.device).view(1, N)
            det = to_np(K.rescore(qp, corpus.prep, ids))[0]
            return det[:, 0], det[:, 1:]
        lv = np.stack([self._scores_at_level(q, cands, l) for l in range(len(ql))], axis=1)
        # per candidate: float32 arithmetic when both arrays are float32 (mixed lengths are rare: host loop)
        out = np.zeros(N)
        q32 = _is_f32(q)
        for both32 in (False, True):
            sel = [i for i, c in enumerate(cands) if (q32 and _is_f32(c)) == both32]
            if sel:
                out[sel] = combine_levels(lv[sel], both32)
        return out, lv

    # ---- searches ------------------------------------------------------------------------------
    @staticmethod
    def _uniform(q, pool) -> bool:
        return all(len(c.hierarchical_indices) == len(q) for c in pool)

    def _results(self, pool, ids, ov, lv, count=None, with_error=True) -> List[SearchResult]:
        out = []
        n = len(ids) if count is None else int(count)
        for j in range(n):
            i = int(ids[j])
            if i < 0:
                break
            sim = float(min(1.0, max(0.0, ov[j])))
            err = max(0.0, 1.0 - float(ov[j])) if with_error else 0.0
            out.append(SearchResult(model=pool[i], similarity_score=sim,
                                    matching_indices={l: float(lv[j, l]) for l in range(lv.shape[1])},
                                    reconstruction_error=err))
        return out

    def brute_force_search(self, query_indices, candidate_pool: List[QuantizedModel],
                           max_results: int) -> List[SearchResult]:
        if len(query_indices) == 0 or not candidate_pool:
            return []
        q = _idx(query_indices)
        if self._uniform(q, candidate_pool):
            corpus = self._pool_corpus(candidate_pool)
            ids, ov, lv = corpus.brute_force(q[None], min(max_results, len(candidate_pool)))
            return self._results(candidate_pool, to_np(ids)[0], to_np(ov)[0], to_np(lv)[0], with_error=False)
        ov, lv = self._overall_many(q, [c.hierarchical_indices for c in candidate_pool])
        order = np.argsort(-ov, kind="stable")[:max_results]
        return self._results(candidate_pool, order, ov[order], lv[order], with_error=False)

    def progressive_search(self, query_indices, candidate_pool: List[QuantizedModel],
                           max_results: int) -> List[SearchResult]:
        if len(query_indices) == 0 or not candidate_pool:
            return []
        q = _idx(query_indices)
        if not self._parse_index_structure(q, len(q)):
            return []
        if self._uniform(q, candidate_pool):
            corpus = self._pool_corpus(candidate_pool)
            ids, ov, lv, cnt = corpus.progressive(q[None], max_results, self.similarity_threshold,
                                                  self.max_candidates_per_level)
            return self._results(candidate_pool, to_np(ids)[0], to_np(ov)[0], to_np(lv)[0], int(to_np(cnt)[0]))
        return self._progressive_mixed(q, candidate_pool, max_results)

    def progressive_search_batch(self, queries: Sequence, candidate_pool: List[QuantizedModel],
                                 max_results: int) -> List[List[SearchResult]]:
        """progressive_search for many queries against one pool: one resident corpus and one batched
        scan when every index has the same length (else query by query)."""
        if not candidate_pool:
            return [[] for _ in queries]
        qs = [_idx(q) for q in queries]
        L = len(qs[0]) if qs else 0
        if not qs or any(len(q) != L for q in qs) or L == 0 or not self._parse_index_structure(qs[0], L) \
                or not self._uniform(qs[0], candidate_pool):
            return [self.progressive_search(q, candidate_pool, max_results) for q in qs]
        corpus = self._pool_corpus(candidate_pool)
        Qa, qflags = _stack_rows(qs)
        ids, ov, lv, cnt = corpus.progressive(Qa if qflags is None else (Qa, qflags), max_results,
                                              self.similarity_threshold,
                                              self.max_candidates_per_level)
        ids, ov, lv, cnt = to_np(ids), to_np(ov), to_np(lv), to_np(cnt)
        return [self._results(candidate_pool, ids[i], ov[i], lv[i], int(cnt[i])) for i in range(len(qs))]

    def _progressive_mixed(self, q, pool, max_results):
        """Candidate pools of mixed index length: scores from the GPU, the reference's level loop
        (:254-300) applied to them."""
        cands = [np.asarray(c.hierarchical_indices) for c in pool]
        nl = len(self._parse_index_structure(q, len(q)))
        cur = np.arange(len(pool))
        prev: Dict[int, np.ndarray] = {}
        for lv in range(nl):
            if len(cur) <= self.max_candidates_per_level:
                break
            s = self._scores_at_level(q, [cands[i] for i in cur], lv)
            now = dict(prev)
            now[lv] = s
            tw = sum(1.0 / (i + 1) for i in now)
            comb = sum(now[i] * (1.0 / (i + 1)) for i in now) / tw
            keep = np.nonzero(s >= self.similarity_threshold)[0]
            if len(keep):
                keep = keep[np.argsort(-comb[keep], kind="stable")][: self.max_candidates_per_level]
            else:
                keep = np.array([int(np.argmax(s))])
            cur = cur[keep]
            prev = {k: v[keep] for k, v in now.items()}
        ov, lvs = self._overall_many(q, [cands[i] for i in cur])
        order = np.argsort(-ov, kind="stable")[:max_results]
        return self._results(pool, cur[order], ov[order], lvs[order])
