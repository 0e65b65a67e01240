#!/usr/bin/env python3
"""Level-0 scan timing experiments: python tools/scan_expt.py [N] [Q]; HQ_SCAN_EXPT / HQ_SCAN_* env
variables select kernel variants.  Prints ms per scan_topk call (k = 28, threshold 0.1)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
g = torch.Generator(device="cuda").manual_seed(5)
if os.environ.get("SCAN_DATA", "bench") == "bench":  # the bench corpus: streaming indexes of N(0,1) embeddings
    X = torch.randn((N, 1536), generator=g, device="cuda", dtype=torch.float32)
    _, C, _ = K.map_index_quantize(X, 64, 64)
    del X
else:  # random walks
    C = torch.randn((N, 64), generator=g, device="cuda", dtype=torch.float64).cumsum(1) * 0.1
corpus = IndexCorpus(C)
qp = corpus.prepare_queries(C[:Q] + 0.01 * torch.randn((Q, 64), generator=g, device="cuda", dtype=torch.float64))
VARIANTS = [("count", {"HQ_SCAN_EXPT": "3"}), ("default", {}),
                  ("no-sample", {"HQ_SCAN_NOSAMPLE": "1"}), ("f64", {"HQ_SCAN_F64": "1"})]
only = os.environ.get("SCAN_EXPT_ONLY")
for name, env in VARIANTS:
    if only and name not in only.split(","):
        continue
    for k, v in env.items():
        os.environ[k] = v
    K.scan_topk(qp, corpus.prep, 0, 28, 0.1, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        K.scan_topk(qp, corpus.prep, 0, 28, 0.1, 1)
    torch.cuda.synchronize()
    print(f"{name:10s} {(time.perf_counter() - t0) / 5 * 1e3:8.3f} ms", flush=True)
    for k in env:
        del os.environ[k]
