#!/usr/bin/env python3
"""Clustered-corpus timing (bench.py's `clustered` mode: 1M rows in 64-row runs of near-duplicates): one
1000-query progressive batch at M = 20 split into its phases (first pass, the longer-list retry of the
unproven queries, their final ranking), wall clock with stream syncs, for a kernel trace under rocprofv3."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402

dev = torch.device("cuda")
N, QN, RUN, d = 1_000_000, 1000, 64, 1536
nb = N // RUN
g = torch.Generator(device=dev).manual_seed(6)
_, B, _ = K.map_index_quantize(torch.randn((nb, d), generator=g, device=dev, dtype=torch.float32), 64, 64)
C = B.repeat_interleave(RUN, 0)
C.add_(0.01 * torch.randn(C.shape, generator=g, device=dev, dtype=torch.float64))
pick = torch.randperm(nb, generator=torch.Generator().manual_seed(7))[:QN].to(dev)
Q = B[pick] + 0.01 * torch.randn((QN, 64), generator=g, device=dev, dtype=torch.float64)
corpus = IndexCorpus(C)
M = int(os.environ.get("HQ_M", "20"))


def wall(f, reps=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


torch.cuda.synchronize()
t0 = time.perf_counter()
corpus.progressive(Q, 10, 0.1, M)
torch.cuda.synchronize()
print(f"cold first batch (process and corpus cold): {(time.perf_counter() - t0) * 1e3:.3f} ms {corpus.stats}", flush=True)
fresh = IndexCorpus(C)  # the bench's case: warm process, a new corpus
torch.cuda.synchronize()
t0 = time.perf_counter()
fresh.progressive(Q, 10, 0.1, M)
torch.cuda.synchronize()
print(f"first batch of a new corpus: {(time.perf_counter() - t0) * 1e3:.3f} ms {fresh.stats}", flush=True)
del fresh
corpus.reset_list_lengths()
print(f"progressive M={M} (the first of 6 calls adapts the list length): "
      f"{wall(lambda: corpus.progressive(Q, 10, 0.1, M)):.3f} ms", flush=True)
corpus.reset_list_lengths()
qp = corpus.prepare_queries(Q)
nredo, nnext, _ = corpus._redo_counter(dev)
out = corpus._scan_refine(qp, 0, M, 0.1, 1, nredo, det=True, next_redo=nnext)
res, cnt = out[3], out[2]
sel = torch.nonzero(res == 0).view(-1)
print(f"unproven after the first pass: {sel.numel()}", flush=True)
print(f"first pass (scan + re-rank): {wall(lambda: corpus._scan_refine(qp, 0, M, 0.1, 1, det=True)):.3f} ms", flush=True)
sub = qp.rows(sel)
print(f"rows(): {wall(lambda: qp.rows(sel)):.3f} ms", flush=True)
print(f"retry scan + re-rank ({sel.numel()} queries, list {corpus.RETRY_FACTOR * (M + corpus.SLACK)}): "
      f"{wall(lambda: corpus._retry_scan(sub, 0, M, 0.1, 1, M + corpus.SLACK, det=True)):.3f} ms", flush=True)
print(f"level0 redo (retry + bookkeeping): "
      f"{wall(lambda: corpus._level0_redo(qp, sel, M, 0.1, res, cnt, None)):.3f} ms", flush=True)
