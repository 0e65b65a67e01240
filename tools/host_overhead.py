#!/usr/bin/env python3
"""Host time of one progressive batch (cfg3, M = 20): wall time inside progressive_submit and
progressive_finish (excluding the wait on the batch's event), against the GPU time per batch, plus a
cProfile of the submits (top functions by own time)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(2)
X = torch.randn((1_000_000, 1536), generator=g, device=dev, dtype=torch.float32)
_, C, _ = K.map_index_quantize(X, 64, 64)
del X
corpus = IndexCorpus(C)
gq = torch.Generator(device=dev).manual_seed(3)
Q = C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device=dev, dtype=torch.float64)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for _ in range(5):
    corpus.progressive_finish(corpus.progressive_submit(Q, 10, 0.1, M))
torch.cuda.synchronize()
n = 50
ts = tf = 0.0
pend = []
t0 = time.perf_counter()
for i in range(n):
    a = time.perf_counter()
    pend.append(corpus.progressive_submit(Q, 10, 0.1, M))
    ts += time.perf_counter() - a
    if len(pend) >= 2:
        p = pend.pop(0)
        p.event.synchronize()
        a = time.perf_counter()
        corpus.progressive_finish(p)
        tf += time.perf_counter() - a
for p in pend:
    corpus.progressive_finish(p)
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"M={M}: wall {wall / n * 1e6:.1f} us/batch, submit {ts / n * 1e6:.1f} us, finish (after the event) {tf / n * 1e6:.1f} us")
pr = cProfile.Profile()
pr.enable()
for i in range(20):
    corpus.progressive_finish(corpus.progressive_submit(Q, 10, 0.1, M))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
