"""Pre-computed index kernel time vs the output row stride (A/B tool, GPU): the 2,610-float rows of a
dense [N, T] output start at 8-byte offsets mod 128 B; padded strides align every row to a cache line."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hilbert-quantization_amd"))
from hq_mi355x import _lib, kernels as K  # noqa: E402
from hq_mi355x._dev import ptr, stream  # noqa: E402

N, d, n = 1_000_000, 1536, 64
dev = torch.device("cuda:0")
X = torch.randn((N, d), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
T = sum(c for (_, _, c, _) in K.precomputed_layout(n))
ref = None
for rep in range(2):
    for ld in (T, T + 2, (T + 3) // 4 * 4, (T + 31) // 32 * 32, (T + 63) // 64 * 64):
        out = torch.empty((N, ld), dtype=torch.float32, device=dev)

        def step():
            _lib.check(_lib.lib().hq_precomputed_index(0, 1, ptr(X), N, d, d, n, 6, 2, ptr(out), ld, stream()))
        step()
        torch.cuda.synchronize()
        if ref is None:
            ref = out[:, :T].clone()
        else:
            assert torch.equal(out[:, :T], ref), ld
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f"stride {ld}: {ms:.3f} ms  frac {(4 * d + 4 * T) * N / ms / 1e6 / 8000:.3f}", flush=True)
        del out
