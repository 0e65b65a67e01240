#!/usr/bin/env python3
"""Diagnostic: how many corpus candidates pass the sampled starting threshold (bench-like corpus)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402
from hq_mi355x.core.search_engine import IndexCorpus  # noqa: E402

N, Kp = 1_000_000, 28
dev = torch.device("cuda")
for kind in ("bench", "walk"):
    g = torch.Generator(device=dev).manual_seed(2)
    if kind == "bench":
        X = torch.randn((N, 1536), generator=g, device=dev, dtype=torch.float32)
        _, C, _ = K.map_index_quantize(X, 64, 64)
        del X
    else:
        C = torch.randn((N, 64), generator=g, device=dev, dtype=torch.float64).cumsum(1) * 0.1
    corpus = IndexCorpus(C)
    Qv = C[:8] + 0.01 * torch.randn((8, 64), generator=g, device=dev, dtype=torch.float64)
    s = corpus.level_scores(Qv, 0)
    for i in range(4):
        row = s[i]
        top = torch.sort(row, descending=True).values
        samp = torch.sort(row[::16], descending=True).values
        kth_s = float(samp[Kp - 1])
        edge = int(kth_s * 256) / 256 - 3e-5
        print(f"{kind} q{i}: true K'th {float(top[Kp-1]):.5f}  sample K'th {kth_s:.5f}  bin edge {edge:.5f}  "
              f"pass@sampleK'th {int((row >= kth_s).sum())}  pass@edge {int((row >= edge).sum())}  "
              f"sample-in-bin {int((row[::16] >= edge).sum())}", flush=True)
