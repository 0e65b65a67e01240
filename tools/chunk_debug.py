#!/usr/bin/env python3
"""cfg5 chunk encoder on a 7e9-value f16 stream (as bench.py's stream leg), three calls, for PMC passes
(tools/pmc_kernel.sh k_chunk_np <outdir> chunk)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]
import torch  # noqa: E402
from hq_mi355x import kernels as K  # noqa: E402

dev = torch.device("cuda")
total = 7_000_000_000
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn((total,), generator=g, device=dev, dtype=torch.float16).mul_(0.02)
nch = (total + 1023) // 1024
out = (torch.zeros((nch, 33, 32), dtype=torch.uint8, device=dev), torch.zeros((nch, 32), dtype=torch.float32, device=dev),
       torch.zeros((nch, 2), dtype=torch.float32, device=dev))
for _ in range(3):
    K.chunk_encode_f16(x, 1024, out=out)
torch.cuda.synchronize()
