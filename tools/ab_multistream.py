"""A/B: one launch vs the same work split over S launches on S HIP streams (hardware queues), for the
cfg5 chunk kernel and the cfg2 fused kernel.  Two ranks sharing one GPU outran one process on the
stream config, which points at per-queue workgroup dispatch, not HBM, as the single-launch limit."""
import sys
import time

import torch

sys.path.insert(0, "hilbert-quantization_amd")
from hq_mi355x import kernels as K  # noqa: E402


def run_split(fn, n, S, reps=10):
    cur = torch.cuda.current_stream()
    streams = [cur] + [torch.cuda.Stream() for _ in range(S - 1)]
    cuts = [n * i // S for i in range(S + 1)]

    def once():
        ev = torch.cuda.Event()
        ev.record(cur)
        for i, st in enumerate(streams):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                fn(cuts[i], cuts[i + 1])
        for st in streams[1:]:
            e2 = torch.cuda.Event()
            e2.record(st)
            cur.wait_event(e2)

    once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    if "--fused-only" in sys.argv:
        return fused(dev)
    nch = 6_835_937
    x = torch.randn((nch * 1024,), device=dev, dtype=torch.float16).mul_(0.02)
    fr = torch.empty((nch, 33, 32), dtype=torch.uint8, device=dev)
    ix = torch.empty((nch, 32), dtype=torch.float32, device=dev)
    mm = torch.empty((nch, 2), dtype=torch.float32, device=dev)
    ref = None
    for S in (1, 2, 4, 1, 2, 4):
        dt = run_split(lambda a, b: K.chunk_encode_f16(x[a * 1024:b * 1024], 1024, out=(fr[a:b], ix[a:b], mm[a:b])), nch, S)
        print(f"stream S={S}: {nch * 3240 / dt / 1e9:.0f} GB/s ({dt * 1e3:.2f} ms)", flush=True)
        if ref is None:
            ref = (fr.clone(), ix.clone(), mm.clone())
        else:
            assert torch.equal(ref[0], fr) and torch.equal(ref[1], ix) and torch.equal(ref[2], mm)
    del x, fr, ix, mm, ref
    fused(dev)


def fused(dev):
    N, d, n, L = 1_000_000, 1536, 64, 64
    if "--pool" in sys.argv:  # one cached segment for all buffers (what the stream test leaves behind)
        big = torch.empty((int(sys.argv[sys.argv.index("--pool") + 1]) << 30,), dtype=torch.uint8, device=dev)
        del big
    X = torch.randn((N, d), device=dev, dtype=torch.float32)
    F = torch.empty((N, n + 1, n), dtype=torch.uint8, device=dev)
    I = torch.empty((N, L), dtype=torch.float64, device=dev)
    M = torch.empty((N, 2), dtype=torch.float32, device=dev)
    print("ptrs X F I M", [hex(t.data_ptr()) for t in (X, F, I, M)], flush=True)
    ref = None
    for S in (1, 1, 2):
        dt = run_split(lambda a, b: K.map_index_quantize(X[a:b], n, L, out=(F[a:b], I[a:b], M[a:b])), N, S)
        print(f"fused S={S}: {N / dt / 1e6:.1f}M emb/s ({N * 10824 / dt / 1e9:.0f} GB/s)", flush=True)
        if ref is None:
            ref = (F.clone(), I.clone(), M.clone())
        else:
            assert torch.equal(ref[0], F) and torch.equal(ref[1], I) and torch.equal(ref[2], M)


if __name__ == "__main__":
    main()
