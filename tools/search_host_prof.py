#!/usr/bin/env python3
"""Host-side cost of IndexCorpus.progressive on the bench corpus: wall time per call and a cProfile of
the Python functions (the GPU idles while the host prepares the first launches after each sync)."""
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
for _ in range(5):
    corpus.progressive(Q, 10, 0.1, 20)
torch.cuda.synchronize()
n = 50
t0 = time.perf_counter()
for _ in range(n):
    corpus.progressive(Q, 10, 0.1, 20)
torch.cuda.synchronize()
print(f"wall per call {1e6 * (time.perf_counter() - t0) / n:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    corpus.progressive(Q, 10, 0.1, 20)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
