#!/usr/bin/env python3
"""Debug counters of the level-0 scan on the bench corpus (HQ_SCAN_EXPT=3)."""
# HQ_SCAN_EXPT=3 counters need the diagnostics build (make -C hilbert-quantization_amd/csrc DIAG=1).
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
os.environ.setdefault("HQ_SCAN_EXPT", "0")
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
qp = corpus.prepare_queries(C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device=dev, dtype=torch.float64))
K.scan_topk(qp, corpus.prep, 0, 28, 0.1 - 2e-5, 1)
torch.cuda.synchronize()
