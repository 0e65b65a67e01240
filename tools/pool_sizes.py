#!/usr/bin/env python3
"""Pool sizes of the level-0 scan (cfg3 corpus, 1000 bench queries) at list lengths 28 / 108 / 1008: the
per-query pool counts read back from the scan workspace (layout of scan0_run: pools, gtau Q x 8, histogram
Q x 256 x 4, pool_n Q x 4), and the per-phase times (scan + pool select/sort, cooperative re-rank)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import numpy as np  # noqa: E402
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
qp = corpus.prepare_queries(Q)
N, Qn = corpus.N, 1000


def kprime(k, stride=16):
    from math import lgamma, exp, log, log1p
    p = 1.0 / stride
    lk = lgamma(k + 1.0)
    tail = 0.0
    for i in range(k, 0, -1):
        tail += exp(lk - lgamma(i + 1.0) - lgamma(k - i + 1.0) + i * log(p) + (k - i) * log1p(-p))
        if tail > 1e-7:
            return min(i + 1, k)
    return 1


for kp in (28, 108, 1008):
    K.scan_topk(qp, corpus.prep, 0, kp, 0.1 - corpus.EPS, 1, 0)
    torch.cuda.synchronize()
    ws = max(K._WS.values(), key=lambda t: t.numel())
    if kp <= 64:
        print(f"kp={kp}: list pools (nchunks x k), not read", flush=True)
        continue
    want = 3 * 16 * kprime(kp) + 1024
    cap = 4096
    while cap < want and cap < (1 << 22):
        cap <<= 1
    cap = min(cap, (N + 63) // 64 * 64)
    lists = (Qn * cap * 8 + 255) & ~255
    off = lists + Qn * 8 + Qn * 256 * 4
    pn = ws[off:off + Qn * 4].view(torch.int32).cpu().numpy()
    print(f"kp={kp}: K'={kprime(kp)} cap={cap} pool_n min/median/p90/max = {pn.min()} {int(np.median(pn))} "
          f"{int(np.percentile(pn, 90))} {pn.max()}, > 4096: {(pn > 4096).sum()}", flush=True)
