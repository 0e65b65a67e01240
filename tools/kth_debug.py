#!/usr/bin/env python3
"""Statistical starting threshold (HQ_SAMPLE_KTH) on the bench corpus: how many queries end unresolved
or empty after the scan + exact re-rank, and the scan lists' fill."""
import os
import sys

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
qp = corpus.prepare_queries(C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device=dev, dtype=torch.float64))
asc, aid, _, _ = K.scan_topk(qp, corpus.prep, 0, 28, 0.1 - 2e-5, 1)
s0, ids, cnt, res = K.refine_topk(qp, corpus.prep, 0, asc, aid, 20, 0.1, 1, 2e-5, count_empty=True)
fill = (aid >= 0).sum(1)
trunc = ((aid[:, -1] < 0) & torch.isinf(asc[:, -1]) & (asc[:, -1] > 0)).sum()
print("kth", os.environ.get("HQ_SAMPLE_KTH"), "unresolved", int((res == 0).sum()), "empty", int((cnt == 0).sum()),
      "truncated", int(trunc), "list fill min/mean", int(fill.min()), float(fill.float().mean()))
