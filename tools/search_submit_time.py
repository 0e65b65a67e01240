#!/usr/bin/env python3
"""Host time of IndexCorpus.progressive_submit / progressive_finish on the bench corpus (cfg3), with two
batches in flight as in bench.py: if submit costs about a batch's GPU time, the host bounds the rate."""
import os
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
for _ in range(5):
    corpus.progressive(Q, 10, 0.1, 20)
torch.cuda.synchronize()
n = 100
ts, tf = 0.0, 0.0
pend = []
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    pend.append(corpus.progressive_submit(Q, 10, 0.1, 20))
    ts += time.perf_counter() - a
    if len(pend) > 1:
        a = time.perf_counter()
        corpus.progressive_finish(pend.pop(0))
        tf += time.perf_counter() - a
while pend:
    corpus.progressive_finish(pend.pop(0))
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"per batch: wall {1e6 * wall / n:.1f} us, submit (host) {1e6 * ts / n:.1f} us, finish (host, incl. wait) "
      f"{1e6 * tf / n:.1f} us")
