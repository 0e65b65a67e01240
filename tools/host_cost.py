"""Host time per progressive batch on the cfg3 workload (M = 20 / 100): submit and finish separately
(perf_counter), pipelined at depth 2 and 3, and the wall time per batch — whether the bench's search leg is
bound by the host's launch path rather than the GPU's kernels."""
import sys, time
sys.path.insert(0, "hilbert-quantization_amd")
import torch
from hq_mi355x import kernels as K
from hq_mi355x.core.search_engine import IndexCorpus

g = torch.Generator(device="cuda").manual_seed(2)
_, C, _ = K.map_index_quantize(torch.randn((1_000_000, 1536), generator=g, device="cuda"), 64, 64)
gq = torch.Generator(device="cuda").manual_seed(3)
Q = C[:1000] + 0.01 * torch.randn((1000, 64), generator=gq, device="cuda", dtype=torch.float64)
corpus = IndexCorpus(C)
for M in (20, 100):
    for depth in (2, 3, 4):
        for _ in range(3):
            corpus.progressive(Q, 10, 0.1, M)
        torch.cuda.synchronize()
        n = 200
        ts = tf = 0.0
        pend = []
        t0 = time.perf_counter()
        for i in range(n):
            a = time.perf_counter()
            pend.append(corpus.progressive_submit(Q, 10, 0.1, M))
            b = time.perf_counter()
            ts += b - a
            if len(pend) >= depth:
                corpus.progressive_finish(pend.pop(0))
                tf += time.perf_counter() - b
        while pend:
            corpus.progressive_finish(pend.pop(0))
        torch.cuda.synchronize()
        w = time.perf_counter() - t0
        print(f"M={M} depth={depth}: wall {w / n * 1e6:.1f} us/batch ({1000 * n / w / 1e6:.3f}M QPS), "
              f"submit {ts / n * 1e6:.1f} us, finish (incl. wait) {tf / n * 1e6:.1f} us", flush=True)
