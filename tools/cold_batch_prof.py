#!/usr/bin/env python3
"""Where the clustered corpus's first (cold) progressive batch spends its time, in the bench's order: a warm
process (cfg3-shaped corpus searched first), the allocator cache emptied (bench.py empties it between legs),
then a new 1M-row corpus of 64-row near-duplicate runs and its first M = 20 batch under cProfile (host time
by function: the syncs and allocations show as the calls that block), then the second batch for comparison."""
import cProfile
import io
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
N, QN, RUN, d = 1_000_000, 1000, 64, 1536
g = torch.Generator(device=dev).manual_seed(2)
_, C0, _ = K.map_index_quantize(torch.randn((N, d), generator=g, device=dev, dtype=torch.float32), 64, 64)
warm = IndexCorpus(C0)
Q0 = C0[:QN] + 0.01 * torch.randn((QN, 64), generator=g, device=dev, dtype=torch.float64)
for M in (20, 100, 1000):
    for _ in range(3):
        warm.progressive(Q0, 10, 0.1, M)
torch.cuda.synchronize()
del warm, C0, Q0
torch.cuda.empty_cache()

nb = N // RUN
g = torch.Generator(device=dev).manual_seed(6)
_, B, _ = K.map_index_quantize(torch.randn((nb, d), generator=g, device=dev, dtype=torch.float32), 64, 64)
C = B.repeat_interleave(RUN, 0)
C.add_(0.01 * torch.randn(C.shape, generator=g, device=dev, dtype=torch.float64))
pick = torch.randperm(nb, generator=torch.Generator().manual_seed(7))[:QN].to(dev)
Q = B[pick] + 0.01 * torch.randn((QN, 64), generator=g, device=dev, dtype=torch.float64)
corpus = IndexCorpus(C)
torch.cuda.synchronize()

for label in ("first batch", "second batch", "third batch"):
    corpus.reset_list_lengths()  # every batch takes the retry (the adapted list would skip it)
    corpus.reset_stats()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    p = corpus.progressive_submit(Q, 10, 0.1, 20)
    t1 = time.perf_counter()
    corpus.progressive_finish(p)
    torch.cuda.synchronize()
    pr.disable()
    t2 = time.perf_counter()
    st = corpus.stats
    print(f"{label}: submit {(t1 - t0) * 1e3:.3f} ms, finish + sync {(t2 - t1) * 1e3:.3f} ms, "
          f"redo stream time {st['dense_s'] * 1e3:.3f} ms, {st}", flush=True)
    if label != "third batch":
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
        print("\n".join(s.getvalue().splitlines()[:40]), flush=True)
