#!/usr/bin/env python3
"""Overall (brute-force) scan check on the cfg3 corpus (1M x L=64, queries = corpus rows + noise and
random rows): the scan + exact re-rank under each bound variant against the dense exact scorer (every
pair), and the scan's raw candidate lists (k + slack) compared between variants."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402
from hq_mi355x import _lib  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(2)
X = torch.randn((1_000_000, 1536), generator=g, device=dev, dtype=torch.float32)
_, C, _ = K.map_index_quantize(X, 64, 64)
del X
corpus = IndexCorpus(C)
gq = torch.Generator(device=dev).manual_seed(3)
Qv = torch.cat([C[:500] + 0.01 * torch.randn((500, 64), generator=gq, device=dev, dtype=torch.float64),
                torch.randn((500, 64), generator=gq, device=dev, dtype=torch.float64)])
qp = corpus.prepare_queries(Qv)
k = 10
ds, di, _, _ = corpus._dense(qp, torch.arange(len(Qv), device=dev), 1, k, 0.0, 0)
di = di.cpu()
res = {}
for tag, opts in (("lin", {}), ("v1", {"scanov_v1": 1})):
    for n, v in opts.items():
        _lib.set_option(n, v)
    asc, aid, _, _ = K.scan_topk(qp, corpus.prep, 1, k + corpus.SLACK, -corpus.EPS, 0, 0)
    sc, ids, cnt, rs = K.refine_topk(qp, corpus.prep, 1, asc, aid, k, 0.0, 0, corpus.EPS, 0)
    torch.cuda.synchronize()
    for n in opts:
        _lib.reset_option(n)
    ids = ids.cpu(); rs = rs.cpu()
    bad = [a for a in range(len(Qv)) if rs[a] and not torch.equal(ids[a], di[a])]
    res[tag] = aid.cpu()
    print(tag, "resolved", int(rs.sum()), "mismatch vs dense", len(bad), bad[:10], flush=True)
A, B = res["lin"], res["v1"]
diff = [a for a in range(len(Qv)) if set(A[a].tolist()) != set(B[a].tolist())]
print("raw candidate lists differ on", len(diff), "queries", diff[:10])
