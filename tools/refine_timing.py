#!/usr/bin/env python3
"""Long-list re-rank timing on the cfg3 corpus (1M x L=64, 1000 queries): the scan list for k + slack,
then hq_refine_topk (ranking only) and hq_refine_rescore_topk (with the [overall, levels] records), at
M = 100 and 1000, CUDA events on the current stream."""
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


def timed(f, reps=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


from hq_mi355x import _lib  # noqa: E402

for M, coop in ((100, 1), (100, 0), (1000, 1), (1000, 0)):
    _lib.set_option("refine_coop", coop)
    kp = M + corpus.SLACK
    asc, aid, _, _ = K.scan_topk(qp, corpus.prep, 0, kp, 0.1 - corpus.EPS, 1, 0)
    t_scan = timed(lambda: K.scan_topk(qp, corpus.prep, 0, kp, 0.1 - corpus.EPS, 1, 0))
    t_ref = timed(lambda: K.refine_topk(qp, corpus.prep, 0, asc, aid, M, 0.1, 1, corpus.EPS, 0))
    t_det = timed(lambda: K.refine_rescore_topk(qp, corpus.prep, 0, asc, aid, M, 0.1, 1, corpus.EPS, 0))
    _, ids, _, _ = K.refine_topk(qp, corpus.prep, 0, asc, aid, M, 0.1, 1, corpus.EPS, 0)
    t_res = timed(lambda: K.rescore(qp, corpus.prep, ids, 0))
    print(f"M={M} coop={coop}: scan+select {t_scan:.1f} us  refine {t_ref:.1f} us  refine+records {t_det:.1f} us  "
          f"rescore of the output {t_res:.1f} us", flush=True)
