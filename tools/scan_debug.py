#!/usr/bin/env python3
"""The level-0 scan on the bench corpus (cfg3 shape: 1M x 64 level-0 values, 1000 queries), three
calls, for PMC passes (tools/pmc_kernel.sh).  Argument: level0 (default, the progressive search's scan)
or overall (the brute-force overall scan), m20 / m100 / m1000 (whole progressive searches at M = 20 / 100 / 1000), scanNNN (the scan alone, list length NNN)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402
from hq_mi355x import _lib  # noqa: E402

for kv in filter(None, os.environ.get("HQ_DBG_OPTS", "").split(",")):  # kernel variants for A/B passes
    name, value = kv.split("=")
    _lib.set_option(name, int(value))

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(2)
X = torch.randn((1_000_000, 1536), generator=g, device=dev, dtype=torch.float32)
_, C, _ = K.map_index_quantize(X, 64, 64)
del X
corpus = IndexCorpus(C)
gq = torch.Generator(device=dev).manual_seed(3)
qp = corpus.prepare_queries(C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device=dev, dtype=torch.float64))
mode = sys.argv[1] if len(sys.argv) > 1 else "level0"
for _ in range(3):
    if mode == "overall":
        K.scan_topk(qp, corpus.prep, 1, 18, -2e-5, 0)
    elif mode in ("m20", "m100", "m1000"):
        corpus.progressive(C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device=dev, dtype=torch.float64),
                           10, 0.1, int(mode[1:]))
    elif mode.startswith("scan"):  # scanNNN: the level-0 scan alone at list length NNN
        K.scan_topk(qp, corpus.prep, 0, int(mode[4:]), 0.1 - 2e-5, 1)
    else:
        K.scan_topk(qp, corpus.prep, 0, 28, 0.1 - 2e-5, 1)
torch.cuda.synchronize()
