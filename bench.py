#!/usr/bin/env python3
"""Benchmark of the MI355X hot path (BASELINE.json configs 2-4).

Headline `value` (BASELINE.json metric, first half): embeddings/sec of the fused Hilbert map +
streaming index + index-row embed + uint8 quantize (hq_map_index_quantize) on 1M x 1536-d float32
embeddings per GPU (config 2, n = 64, L = 64, min_efficiency_ratio = 0.2), inputs resident in HBM.
A step = one launch over the whole 1M batch.  Weak scaling: every rank processes its own 1M batch.

Second half of the metric, reported in "search": queries/sec @ top-10 of the reference's
progressive search (threshold 0.1, max_candidates_per_level 20 as HilbertQuantizer sets it) over a
1M-frame corpus per GPU (config 3; config 4 = 1M per GPU x N GPUs with the RCCL all-gather merge).

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0          # measured float4 copy on MI355X (MI355X_MICROARCH.md): the practical ceiling


def hbm_roofline(achieved: float, traffic, **extra) -> dict:
    """HBM roofline record: frac against the spec peak, plus the fraction of the measured copy rate."""
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "measured_copy_peak": HBM_COPY_GBS, "frac_of_measured_copy": achieved / HBM_COPY_GBS}
    r.update(extra)
    return r


FP16_MATRIX_PEAK_TFS = 2500.0  # MI355X dense FP16/BF16 MFMA peak (MI355X_MICROARCH.md)
FP64_MATRIX_PEAK_TFS = 78.6    # MI355X FP64 matrix peak (spec, SURVEY.md §8d / BASELINE.md §3)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-emb", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=1536)
    ap.add_argument("--corpus", type=int, default=1_000_000)
    ap.add_argument("--corpus-total", type=int, default=8_000_000,
                    help="cfg4 strong scaling: one global corpus of this many rows, shard_range over the ranks (0: off)")
    ap.add_argument("--queries", type=int, default=1000)
    # 50 batches: the pipeline's fill and drain (one batch's host submit, the last batch's wait) stay ~2% of
    # the timed region (at 20 they were ~5%: 201 us per step against 190 us of kernels per batch)
    ap.add_argument("--search-steps", type=int, default=200)
    ap.add_argument("--no-search", action="store_true")
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--no-precomputed", action="store_true")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--no-frames", action="store_true")
    ap.add_argument("--no-frames-f64", action="store_true", help="skip the f64-score sub-record of the frames leg")
    ap.add_argument("--no-hard", action="store_true", help="skip the fresh / clustered query-distribution search modes")
    ap.add_argument("--no-api", action="store_true", help="skip the drop-in API per-call latency leg")
    ap.add_argument("--no-modes", action="store_true", help="skip the overall / level0 / m100 / m1000 search modes")
    ap.add_argument("--frames", type=int, default=250_000)
    ap.add_argument("--ingest-models", type=int, default=20000)
    ap.add_argument("--stream-values", type=int, default=7_000_000_000)
    ap.add_argument("--stream-steps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--option", action="append", default=[],
                    help="name=value: select a kernel variant (hq_set_option; A/B runs only)")
    ap.add_argument("--py-set", action="append", default=[],
                    help="module:attribute=value (int, or str where the attribute is one; attribute may be Class.attr): "
                         "a host-side variant, e.g. hq_mi355x.kernels:FINAL_LEVEL0_LISTS=1 "
                         "(A/B runs only)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the N > 1 path on a one-GPU box: every rank on one device, gloo collectives
    # (RCCL refuses two ranks on one GPU); the driver's multi-GPU runs use neither
    if os.environ.get("HQ_BENCH_SAME_DEVICE"):
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("HQ_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# batches of a pipelined progressive search in flight (progressive_submit / progressive_finish): with 2, the
# host's submit of batch i + 2 started only once batch i was finished and left the GPU idle at times (M = 20:
# 173 vs 165 us per batch in profiles/r06_ab_count_kernel.txt's host cost rows; 5.70-5.73M vs 5.76-5.77M QPS
# in the bench leg, r06_ab_search_depth.txt); 3 keeps one batch queued behind the running one.
# HQ_SEARCH_DEPTH: A/B knob
SEARCH_DEPTH = int(os.environ.get("HQ_SEARCH_DEPTH", "3"))


def timed(fn, steps, warmup, world, drain=None):
    """drain: completes work fn left in flight (pipelined legs); called after warmup and inside the
    timed region after the last step."""
    for _ in range(warmup):
        fn()
    if drain is not None:
        drain()
    barrier(world)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        fn()
    if drain is not None:
        drain()
    ev1.record()
    barrier(world)
    wall = time.perf_counter() - t0
    return max_over_ranks(wall, world), ev0.elapsed_time(ev1) / 1e3 / steps


def load_traffic(name):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (tools/pmc_traffic.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            rec = json.load(f).get(name)
    except (OSError, ValueError):
        return None
    if not isinstance(rec, dict):
        return None
    return rec.get("hbm_bytes_per_launch")


def cpu_baseline_quantize(dim, seconds):
    """The NumPy oracle (oracle/hq_oracle.py, a restatement of the reference) on host cores."""
    from oracle import hq_oracle as O
    rng = np.random.default_rng(1)
    n = O.optimal_dimensions(dim)[0]
    B = 256
    P = rng.standard_normal((B, dim)).astype(np.float32)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        img = O.map_to_2d(O.pad_parameters(P, n), n)
        idx = O.streaming_index(O.map_from_2d(img), n)
        O.normalize_u8(O.embed_index_row(img, idx))
        done += B
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "embeddings/sec", "cores": 1, "kind": "port",
            "sample": f"{done} x {dim}-d f32 embeddings through oracle map+streaming index+embed+u8 normalise "
                      f"(NumPy, single thread) in {dt:.1f}s"}


def _cpu_worker(job):
    """One host process of the multi-core CPU baseline: the NumPy oracle for `seconds`, count returned."""
    kind, dim, seconds, seed = job
    from oracle import hq_oracle as O
    rng = np.random.default_rng(seed)
    done, t0 = 0, time.perf_counter()
    if kind == "quantize":
        n = O.optimal_dimensions(dim)[0]
        P = rng.standard_normal((64, dim)).astype(np.float32)
        while time.perf_counter() - t0 < seconds:
            img = O.map_to_2d(O.pad_parameters(P, n), n)
            idx = O.streaming_index(O.map_from_2d(img), n)
            O.normalize_u8(O.embed_index_row(img, idx))
            done += len(P)
    else:  # search: progressive top-10 of single queries over a 20k-row L = 64 corpus (candidates scored)
        C = rng.standard_normal((20_000, 64))
        while time.perf_counter() - t0 < seconds:
            O.progressive_search(C[done % 100] + 0.01, C, 10, 0.1, 20)
            done += len(C)
    return done


def cpu_baseline_parallel(dim, seconds):
    """the vectorised NumPy oracle in one process per host core (the box's CPU
    share, at most 16), run BEFORE the GPU is initialised (fork-safe).  Returns rates for the map +
    quantize leg (embeddings/sec) and the progressive search (candidate scores/sec -> queries/sec over
    a 1M corpus)."""
    import multiprocessing as mp
    workers = max(1, min(16, os.cpu_count() or 1))
    out = {}
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        for kind in ("quantize", "search"):
            t0 = time.perf_counter()
            counts = pool.map(_cpu_worker, [(kind, dim, seconds, 100 + w) for w in range(workers)])
            out[kind] = (sum(counts) / (time.perf_counter() - t0), workers)
    return out


def cpu_baseline_quantize_loops(dim, seconds):
    """the reference-SHAPED single-core port (oracle/hq_loops.py: per-element
    coordinate, scatter / gather and streaming-tree loops, as core/hilbert_mapper.py:17-205 and
    core/streaming_index_builder.py:45-243 run them)."""
    from oracle import hq_loops as HL
    from oracle import hq_oracle as O
    rng = np.random.default_rng(1)
    n = O.optimal_dimensions(dim)[0]
    P = rng.standard_normal((64, dim)).astype(np.float32)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        HL.quantize_one(P[done % 64], n, 64)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "embeddings/sec", "cores": 1, "kind": "port",
            "sample": f"{done} x {dim}-d f32 embeddings through the reference-shaped per-element port (oracle/hq_loops.py: "
                      f"pad, per-cell d2xy + scatter, gather, per-value streaming tree, embed, u8 normalise) in {dt:.1f}s",
            "structure": "reference-shaped (per-element Python loops, BASELINE.md §3 item 1)"}


def cpu_baseline_precomputed(dim, seconds):
    """The pre-computed index leg on one host core: the reference-shaped port (oracle/hq_loops.py:
    per-cell map, one np.mean per square) and the vectorised oracle (hq_oracle.precomputed_index over a
    256-embedding batch, one np.mean per square across the batch)."""
    from oracle import hq_loops as HL
    from oracle import hq_oracle as O
    rng = np.random.default_rng(1)
    n = O.optimal_dimensions(dim)[0]
    P = rng.standard_normal((256, dim)).astype(np.float32)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds / 2:
        HL.precomputed_one(P[done % 256], n)
        done += 1
    dt = time.perf_counter() - t0
    res = {"value": done / dt, "unit": "embeddings/sec", "cores": 1, "kind": "port",
           "sample": f"{done} x {dim}-d f32 embeddings through the reference-shaped port (oracle/hq_loops.py "
                     f"precomputed_one: per-cell map, one np.mean per square, 2,610 squares) in {dt:.1f}s",
           "structure": "reference-shaped (per-square loop, core/precomputed_hilbert_index.py:65-212)"}
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds / 2:
        O.precomputed_index(O.map_to_2d(O.pad_parameters(P, n), n))
        done += len(P)
    dt = time.perf_counter() - t0
    res["vectorised"] = {"value": done / dt, "unit": "embeddings/sec", "cores": 1, "kind": "port",
                         "sample": f"{done} x {dim}-d f32 embeddings, oracle map_to_2d + precomputed_index "
                                   f"(NumPy, 256-embedding batches, single thread) in {dt:.1f}s"}
    return res


def cpu_baseline_search_loops(C, Q, seconds):
    """Reference-shaped search: the per-candidate Python loop of core/search_engine.py:232-388 (both level
    structures re-parsed per comparison) over a 10k-row slice, extrapolated linearly to 1M rows."""
    from oracle import hq_loops as HL
    C = C[:10_000]
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < len(Q):
        HL.progressive_search(Q[done], C, 10, 0.1, 20)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done * len(C) / dt / 1_000_000, "unit": "queries/sec over a 1M corpus (extrapolated)",
            "cores": 1, "kind": "port", "candidate_scores_per_sec": done * len(C) / dt,
            "sample": f"{done} queries x {len(C)} candidates through the reference-shaped candidate loop "
                      f"(oracle/hq_loops.py) in {dt:.1f}s, linear in corpus size",
            "structure": "reference-shaped (per-candidate Python loop, BASELINE.md §3 item 1)"}


def cpu_baseline_mode(mode, C, Q, seconds):
    """Vectorised oracle (one core) for the other cfg3 modes: brute-force overall top-10 / strict level-0 scan."""
    from oracle import hq_oracle as O
    C = C[:20_000]
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < len(Q):
        if mode == "overall":
            O.brute_force_search(Q[done], C, 10)
        else:
            O.hierarchical_frame_search(Q[done], C, 10, 0.1)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done * len(C) / dt / 1_000_000, "unit": "queries/sec over a 1M corpus (extrapolated)",
            "cores": 1, "kind": "port",
            "sample": f"{done} queries x {len(C)} candidates, oracle {'brute_force_search' if mode == 'overall' else 'hierarchical_frame_search'} "
                      f"(NumPy, single thread) in {dt:.1f}s, linear in corpus size"}


def cpu_baseline_search(C, Q, seconds):
    from oracle import hq_oracle as O
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < len(Q):
        O.progressive_search(Q[done], C, 10, 0.1, 20)
        done += 1
    dt = time.perf_counter() - t0
    cand_per_s = done * len(C) / dt
    return {"value": cand_per_s / 1_000_000, "unit": "queries/sec over a 1M corpus (extrapolated)",
            "cores": 1, "kind": "port",
            "sample": f"{done} queries x {len(C)} candidates, oracle progressive_search (NumPy, single thread) "
                      f"in {dt:.1f}s, linear in corpus size"}


def bench_precomputed(args, X, world):
    """the pre-computed overlapping-square index HilbertQuantizer.quantize builds per
    model (api.py:162-173, core/precomputed_hilbert_index.py:65-212), batched over the cfg2 embeddings:
    pad + Hilbert map in LDS, 2,610 float32 square averages per 64x64 image (hq_precomputed_index)."""
    from hq_mi355x import kernels as K
    N, d = X.shape
    n = 64
    lay = K.precomputed_layout(n)
    T = sum(c for (_, _, c, _) in lay)
    out = torch.empty((N, T), dtype=torch.float32, device=X.device)
    stride = X.stride(0)

    def step():
        from hq_mi355x import _lib
        from hq_mi355x._dev import ptr, stream
        _lib.check(_lib.lib().hq_precomputed_index(0, 1, ptr(X), N, stride, d, n, 6, 2, ptr(out), T, stream()))

    wall, kern = timed(step, max(2, args.steps // 4), 1, world)
    steps = max(2, args.steps // 4)
    per = 4 * d + 4 * T
    achieved = per * N / kern / 1e9
    del out
    return {"metric": "embeddings/sec pre-computed square-average index (1536D -> 64x64, 2,610 averages)",
            "value": N * world * steps / wall, "unit": "embeddings/sec", "steps": steps,
            "ms_per_step": wall / steps * 1e3, "scaling": "weak",
            "roofline": hbm_roofline(achieved, load_traffic("k_precomp"), algorithmic_bytes_per_embedding=per,
                                     kernel_ms=kern * 1e3)}


def bench_frames(args, world, rank, dev):
    """S7 / north star "frame similarity as a batched dot over N x (side x side) images": 1000 query
    frames against a resident corpus of 64x64 frames (K = 4096) per GPU, (cos + 1) / 2 for every pair
    (rag/search/engine.py:622-660), split-f16 MFMA contraction (hq_cos_scores_mfma).  A step =
    prepare the query batch + score it against the whole corpus (f64 [Q, N] out)."""
    from hq_mi355x import kernels as K
    Nf, Qn, Kd = args.frames, args.queries, 4096
    g = torch.Generator(device=dev).manual_seed(7 + 1000 * rank)
    F = torch.randn((Nf, Kd), generator=g, device=dev, dtype=torch.float32)
    Qf = F[:Qn] + 0.1 * torch.randn((Qn, Kd), generator=g, device=dev, dtype=torch.float32)
    corpus = K.cos_prepare(F)
    del F
    torch.cuda.synchronize()

    def step():  # float32 scores: the reference's own score dtype (rag/search/engine.py computes in float32)
        K.cosine_scores_mfma(K.cos_prepare(Qf), corpus, f32=True)

    def step64():
        K.cosine_scores_mfma(K.cos_prepare(Qf), corpus)

    steps = max(2, args.search_steps)
    wall, kern = timed(step, steps, 1, world)
    flops = 2.0 * Qn * Nf * Kd
    peak = FP16_MATRIX_PEAK_TFS / 3.0
    res = {"metric": "frame-pair cosine scores/sec (1000 queries x 64x64 frames)",
           "value": Qn * Nf * world * steps / wall, "unit": "pairs/sec", "queries": Qn, "frames_per_gpu": Nf,
           "K": Kd, "steps": steps, "ms_per_step": wall / steps * 1e3, "scaling": "weak",
           "scores": "float32 (hq_cos_scores_mfma_f32)",
           "roofline": {"bound": "mfma", "achieved": flops / kern / 1e12, "peak": peak, "unit": "TFLOP/s",
                        "frac": flops / kern / 1e12 / peak, "traffic": load_traffic("k_cos_t"),
                        "note": "algorithmic 2*Q*N*K f32 dot flops per step; peak = dense f16 MFMA / 3 (split-f16: "
                                "hi.hi + hi.lo + lo.hi); traffic = HBM bytes per k_cos_t launch (PMC)"}}
    if not args.no_frames_f64:
        w64, k64 = timed(step64, steps, 1, world)
        res["f64_scores"] = {"value": Qn * Nf * world * steps / w64, "unit": "pairs/sec",
                             "ms_per_step": w64 / steps * 1e3, "frac": flops / k64 / 1e12 / peak}
    del corpus, Qf
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import hq_oracle as O
        rng = np.random.default_rng(7)
        B = rng.standard_normal((20000, Kd)).astype(np.float32)
        A = rng.standard_normal((4, Kd)).astype(np.float32)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < args.cpu_seconds / 4:
            O.rag_cosine(A[n % 4], B)
            n += 1
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": n * len(B) / dt, "unit": "pairs/sec", "cores": 1, "kind": "port",
                               "sample": f"{n} queries x {len(B)} 4096-d frames, oracle rag_cosine (NumPy) in "
                                         f"{dt:.1f}s"}
    return res


def bench_ingest(args):
    """HilbertQuantizer-semantics model ingest (QuantizedModel objects with JPEG
    payloads, registry, pre-computed index) for many 1024-d vectors — BatchQuantizer.quantize_batch
    (one fused launch + one pre-computed-index launch, host JPEG on a thread pool) against the
    per-model drop-in path HilbertQuantizer.quantize on a sample."""
    import contextlib
    import io
    try:
        import PIL  # noqa: F401
    except ImportError:
        return {"skipped": "PIL not importable"}
    from hq_mi355x.api import BatchQuantizer, HilbertQuantizer
    rng = np.random.default_rng(11)
    M = args.ingest_models
    sets = list(rng.standard_normal((M, 1024)).astype(np.float32))
    bq = BatchQuantizer()
    bq.quantize_batch(sets[:64])  # warm-up (library, PIL, thread pool)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bq.quantize_batch(sets)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    hq = HilbertQuantizer()
    S = 100
    with contextlib.redirect_stdout(io.StringIO()):
        hq.quantize(sets[0], model_id="w")
        t1 = time.perf_counter()
        for i in range(S):
            hq.quantize(sets[i], model_id=f"s{i}")
        ds = time.perf_counter() - t1
    res = {"metric": "QuantizedModels/sec ingest (1024-d, JPEG payload + pre-computed index, HilbertQuantizer semantics)",
           "value": M / dt, "unit": "models/sec", "models": M, "seconds": dt,
           "per_model_path": {"value": S / ds, "unit": "models/sec", "sample": f"{S} x HilbertQuantizer.quantize"},
           "note": "host-bound: the JPEG codec (PIL, SURVEY §8f row 2) runs on host threads"}
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_ingest(sets, hq.compression_quality, args.cpu_seconds / 4)
    return res


def cpu_baseline_ingest(sets, quality, seconds):
    """One host core, one model at a time, reference-shaped: per-cell map + streaming tree + u8 normalise
    (oracle/hq_loops.py quantize_one), the same PIL JPEG encode, and the per-square pre-computed index
    (hq_loops.precomputed_one) — the work HilbertQuantizer.quantize does per model (api.py:98-173)."""
    from hq_mi355x.core.compressor import encode_jpeg
    from oracle import hq_loops as HL
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        p = sets[done % len(sets)]
        encode_jpeg(HL.quantize_one(p, 32, 32), quality)
        HL.precomputed_one(p, 32)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "models/sec", "cores": 1, "kind": "port",
            "sample": f"{done} x 1024-d models: reference-shaped map + streaming index + u8 normalise, PIL JPEG, "
                      f"per-square pre-computed index (oracle/hq_loops.py), single thread, {dt:.1f}s",
            "structure": "reference-shaped (per-element / per-square loops, BASELINE.md §3 item 1)"}


STREAM_CHUNK = 1024
STREAM_BYTES_PER_CHUNK = 2 * STREAM_CHUNK + 33 * 32 + 4 * 32 + 8  # f16 in; u8 33x32 frame, f32[32] index, min/max out


def bench_stream(args, world, rank, dev):
    """Config 5: a 7e9-value f16 parameter stream cut into 1024-value chunks (core/streaming_processor.py:
    539-582), each chunk Hilbert-mapped to 32x32, traditional index (L = 32) embedded, uint8 quantized
    (:877-913; hq_chunk_encode_f16).  The chunk range is split into contiguous per-rank shards (strong
    scaling, no collective); the 512-value tail chunk goes to the last rank."""
    from hq_mi355x import kernels as K
    total = args.stream_values
    nch_all = (total + STREAM_CHUNK - 1) // STREAM_CHUNK
    c0, c1 = rank * nch_all // world, (rank + 1) * nch_all // world
    vals = min(c1 * STREAM_CHUNK, total) - c0 * STREAM_CHUNK
    nch = c1 - c0
    g = torch.Generator(device=dev).manual_seed(5 + 1000 * rank)
    x = torch.randn((vals,), generator=g, device=dev, dtype=torch.float16).mul_(0.02)
    out = (torch.zeros((nch, 33, 32), dtype=torch.uint8, device=dev),
           torch.zeros((nch, 32), dtype=torch.float32, device=dev),
           torch.zeros((nch, 2), dtype=torch.float32, device=dev))

    def step():
        K.chunk_encode_f16(x, STREAM_CHUNK, out=out)

    wall, kern = timed(step, args.stream_steps, 1, world)
    alg_bytes = 2 * total + nch_all * (STREAM_BYTES_PER_CHUNK - 2 * STREAM_CHUNK)
    rank_bytes = 2 * vals + nch * (STREAM_BYTES_PER_CHUNK - 2 * STREAM_CHUNK)
    achieved = rank_bytes / kern / 1e9
    res = {
        "metric": "GB/s streaming Hilbert quantize of a 7e9-value f16 parameter stream (algorithmic bytes)",
        "value": alg_bytes * args.stream_steps / wall / 1e9, "unit": "GB/s",
        "params_per_sec": total * args.stream_steps / wall, "values_total": total, "chunks_total": nch_all,
        "values_per_rank": vals, "steps": args.stream_steps, "ms_per_step": wall / args.stream_steps * 1e3,
        "scaling": "strong", "dtype": "f16 in, f32 arithmetic, u8 frames",
        "config": "cfg5: 1024-value chunks -> 32x32 Hilbert image + traditional index (L=32, f32) + u8 33x32 frame, "
                  f"contiguous chunk shards over {world} GPU(s)",
        "roofline": hbm_roofline(achieved, load_traffic("k_chunk_np32"),
                                 algorithmic_bytes_per_chunk=STREAM_BYTES_PER_CHUNK, kernel_ms=kern * 1e3),
    }
    del x, out
    return res


def cpu_baseline_stream(seconds):
    """Oracle chunk encoder (map + traditional index + embed + u8 normalise per 1024-value chunk)."""
    from oracle import hq_oracle as O
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(STREAM_CHUNK * 256) * 0.02).astype(np.float16)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for c in range(256):
            img = O.map_to_2d(x[c * STREAM_CHUNK:(c + 1) * STREAM_CHUNK].astype(np.float32), 32)
            O.normalize_u8(O.embed_index_row(img, O.traditional_index(img, 32)))
        done += 256
    dt = time.perf_counter() - t0
    return {"value": done * STREAM_BYTES_PER_CHUNK / dt / 1e9, "unit": "GB/s (algorithmic bytes)",
            "params_per_sec": done * STREAM_CHUNK / dt, "cores": 1, "kind": "port",
            "sample": f"{done} chunks of 1024 f16 values through the oracle chunk encoder (NumPy, single thread) "
                      f"in {dt:.1f}s"}


def bench_search_strong(args, world, rank, dev):
    """Config 4 as BASELINE.json names it: ONE global 8M-frame corpus (L = 64 index vectors of seed-4
    embeddings, generated 1M rows at a time exactly as tests/test_gpu_fullsize.py::test_cfg4_full_size_8_shards
    builds it), each rank holding its shard_range of the rows (strong scaling: N = 1 answers the whole 8M
    corpus on one GPU), the cfg3 query batch (global rows 0..999 + N(0, 0.01), seed 3), progressive top-10,
    the per-shard records merged after one all-gather (hq_allgather_topk over RCCL at N > 1)."""
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus, shard_range
    Nt, Qn, per = args.corpus_total, args.queries, 1_000_000
    a, b = shard_range(Nt, rank, world)
    C = torch.empty((b - a, 64), dtype=torch.float64, device=dev)
    Q = None
    g = torch.Generator(device=dev).manual_seed(4)
    Xc = torch.empty((per, args.dim), device=dev, dtype=torch.float32)
    t0 = time.perf_counter()
    for j in range((Nt + per - 1) // per):
        r0, r1 = j * per, min(Nt, (j + 1) * per)
        torch.randn((r1 - r0, args.dim), generator=g, out=Xc[: r1 - r0])  # every rank draws the same stream
        lo, hi = max(a, r0), min(b, r1)
        if lo < hi or j == 0:
            _, blk, _ = K.map_index_quantize(Xc[: r1 - r0], 64, 64)
            if j == 0:
                gq = torch.Generator(device=dev).manual_seed(3)
                Q = blk[:Qn] + 0.01 * torch.randn((Qn, 64), generator=gq, device=dev, dtype=torch.float64)
            if lo < hi:
                C[lo - a:hi - a] = blk[lo - r0:hi - r0]
            del blk
    del Xc
    comm = None
    if world > 1:
        if os.environ.get("HQ_BENCH_BACKEND", "nccl") == "nccl":
            from hq_mi355x.rccl import Communicator
            comm = Communicator.from_process_group()
        engine = ShardedIndexCorpus(C, id_base=a, n_total=Nt, comm=comm)
    else:
        engine = IndexCorpus(C)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    pend = []

    def run():
        pend.append(engine.progressive_submit(Q, 10, 0.1, 20))
        if len(pend) >= SEARCH_DEPTH:
            engine.progressive_finish(pend.pop(0))

    def drain():
        while pend:
            engine.progressive_finish(pend.pop(0))

    steps = max(2, args.search_steps)
    wall, kern = timed(run, steps, 1, world, drain)
    ids, ov, _, cnt = engine.progressive(Q, 10, 0.1, 20)
    ids_h = ids.cpu().numpy()
    res = {"metric": "queries/sec@top-10 over the 8M-frame cfg4 corpus (strong scaling)",
           "value": Qn * steps / wall, "unit": "queries/sec", "scaling": "strong", "corpus_total": Nt,
           "corpus_this_rank": b - a, "ranks": world, "queries": Qn, "steps": steps,
           "ms_per_step": wall / steps * 1e3, "build_s": build_s,
           "self_match_rate": float((ids[:, 0].cpu() == torch.arange(Qn)).float().mean()),
           "ids_checksum": int((ids_h.astype(np.int64) * (np.arange(ids_h.size).reshape(ids_h.shape) % 7919 + 1)).sum()),
           "data": "8M x 1536-d N(0,1) embeddings (torch seed 4, 1M-row blocks) -> fused map + streaming index (L=64)",
           "roofline": {"bound": "mfma", "achieved": 2.0 * Qn * (b - a) * 32 / kern / 1e12,
                        "peak": FP16_MATRIX_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": 2.0 * Qn * (b - a) * 32 / kern / 1e12 / FP16_MATRIX_PEAK_TFS,
                        "note": "this rank's level-0 contraction flops (one f16 pass, 2*Q*N*32) per step / step time"}}
    if comm is not None:
        x = torch.zeros((Qn, 21, 3 + engine.local.nseg), dtype=torch.float64, device=dev)
        _, ak = timed(lambda: comm.all_gather(x), 20, 3, world)
        res["allgather"] = {"ms": ak * 1e3, "bytes_per_rank": x.numel() * 8, "ranks": world,
                            "path": "hq_allgather_topk (ncclAllGather over xGMI)"}
    del engine, C, Q
    torch.cuda.empty_cache()
    return res


def summary(rec) -> dict:
    """Every leg's rate and roofline fraction in a few hundred bytes (the full records precede it)."""
    def r3(x):
        return None if x is None else float(f"{x:.4g}")

    def leg(d):
        if not isinstance(d, dict) or "value" not in d:
            return None
        rf = d.get("roofline") or {}
        return [r3(d["value"]), d.get("unit", "").replace("queries/sec", "qps").replace("embeddings/sec", "emb/s"),
                r3(rf.get("frac"))]

    out = {"headline": leg(rec)}
    s = rec.get("search")
    if isinstance(s, dict):
        out["search_m20"] = leg(s)
        for k, v in (s.get("modes") or {}).items():
            if isinstance(v, dict) and "value" in v:
                out[k] = leg(v)
            elif isinstance(v, dict):  # fresh / clustered: QPS per list length
                out[k] = {m: r3(x["value"]) for m, x in v.items() if isinstance(x, dict) and "value" in x}
                wb = (v.get("m20") or {}).get("warmup_batch")
                if wb:
                    out[k]["m20_first_batch_ms"] = r3(wb.get("wall_ms"))
        out["strong_cfg4"] = leg(s.get("strong"))
    for k in ("frames", "precomputed", "stream", "ingest"):
        if k in rec:
            out[k] = leg(rec[k])
    return out


def progressive_rate(engine, Q, M, steps, world, k=10, threshold=0.1):
    """Pipelined progressive search of one query batch per step (SEARCH_DEPTH batches in flight, as the cfg3 leg),
    with the engine's redo counters (IndexCorpus.stats) over the timed batches: queries re-scanned with a
    longer list after a near-tie / short list, queries left for the dense exact path, and the stream time of
    that redo work per batch (between two events around it: IndexCorpus.stats dense_s); the warm-up batch
    also with its host wall time (submit to finished redo)."""
    pend = []

    def run():
        pend.append(engine.progressive_submit(Q, k, threshold, M))
        if len(pend) >= SEARCH_DEPTH:
            engine.progressive_finish(pend.pop(0))

    def drain():
        while pend:
            engine.progressive_finish(pend.pop(0))

    engine.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()  # warm-up batch (first-call allocations, the adaptive list length), then counters from zero
    drain()
    first = dict(engine.stats)  # (waits for the batch's redo)
    first_wall = time.perf_counter() - t0
    engine.reset_stats()
    wall, kern = timed(run, steps, 0, world, drain)
    st = dict(engine.stats)
    nb = max(1, st["batches"])
    Qn = int(Q.shape[0])
    return {"value": Qn * steps / wall, "unit": "queries/sec", "steps": steps, "ms_per_step": wall / steps * 1e3,
            "max_candidates_per_level": M, "batches": st["batches"], "redo_batches": st["redo_batches"],
            "redo_queries": st["redo_queries"], "redo_queries_per_batch": st["redo_queries"] / nb,
            "retry_queries_per_batch": st["retry_queries"] / nb, "dense_queries_per_batch": st["dense_queries"] / nb,
            "redo_ms_per_batch": st["dense_s"] / nb * 1e3,
            "warmup_batch": {"redo_queries": first["redo_queries"], "retry_queries": first["retry_queries"],
                             "dense_queries": first["dense_queries"], "redo_ms": first["dense_s"] * 1e3,
                             "wall_ms": first_wall * 1e3},
            "first_pass_list": M + engine.slack_for(M)}


def dense_one_query_ms(engine, Q, M, reps=3):
    """Wall time of the dense exact path (every pair's level-0 score + exact top-M select + arg-max) for ONE
    query: the cost of one redo."""
    t = torch
    qp = engine.prepare_queries(Q[:1])
    sel = t.zeros(1, dtype=t.int64, device=Q.device)
    engine._dense(qp, sel, 0, M, 0.1, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        engine._dense(qp, sel, 0, M, 0.1, 1)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def bench_search_hard(args, engine, dev, n, L, world):
    """Query distributions without a planted near-duplicate: the cfg3 corpus answered
    for FRESH queries (index vectors of 1000 new seed-5 N(0,1) embeddings: the top-10 sit in the bulk of the
    score distribution), and a CLUSTERED corpus (1M rows in 64-row runs of near-duplicates: 15,625 seed-6
    base vectors + N(0, 0.01), queries = 1000 runs' bases + N(0, 0.01)), where one sampled tile can hold
    16 of a query's 64 best rows.  Per mode and list length: QPS, the queries that took the dense exact
    path (short or unproven lists) and its time, and the one-query redo cost."""
    from hq_mi355x import kernels as K
    from hq_mi355x.core.search_engine import IndexCorpus
    Qn, d = args.queries, args.dim
    steps = max(2, args.search_steps // 2)
    out = {}
    gf = torch.Generator(device=dev).manual_seed(5)
    Xf = torch.randn((Qn, d), generator=gf, device=dev, dtype=torch.float32)
    _, Qf, _ = K.map_index_quantize(Xf, n, L)
    del Xf
    fresh = {}
    for M in (20, 100, 1000):
        fresh[f"m{M}"] = progressive_rate(engine, Qf, M, steps, world)
    fresh["dense_one_query_ms"] = {f"m{M}": dense_one_query_ms(engine, Qf, M) for M in (20, 100, 1000)}
    fresh["queries"] = "fused-kernel index vectors (L=64) of 1000 fresh N(0,1) 1536-d embeddings (torch seed 5)"
    out["fresh"] = fresh
    Nc = args.corpus
    run = 64
    nb = (Nc + run - 1) // run
    gc = torch.Generator(device=dev).manual_seed(6)
    Xb = torch.randn((nb, d), generator=gc, device=dev, dtype=torch.float32)
    _, B, _ = K.map_index_quantize(Xb, n, L)
    del Xb
    C = B.repeat_interleave(run, 0)[:Nc]
    C.add_(0.01 * torch.randn(C.shape, generator=gc, device=dev, dtype=torch.float64))
    pick = torch.randperm(nb, generator=torch.Generator().manual_seed(7))[:Qn].to(dev)
    Qc = B[pick] + 0.01 * torch.randn((Qn, L), generator=gc, device=dev, dtype=torch.float64)
    del B
    ce = IndexCorpus(C)
    torch.cuda.synchronize()
    clus = {}
    for M in (20, 100, 1000):
        clus[f"m{M}"] = progressive_rate(ce, Qc, M, steps, world)
    ids, _, _, _ = ce.progressive(Qc, 10, 0.1, 20)
    clus["top1_in_own_run"] = float(((ids[:, 0] // run) == pick).float().mean())
    clus["corpus"] = (f"{Nc} rows = {nb} seed-6 base index vectors x {run}-row runs + N(0, 0.01); queries = 1000 "
                      "random runs' bases + N(0, 0.01)")
    out["clustered"] = clus
    del ce, C, Qc
    torch.cuda.empty_cache()
    return out


def bench_api(args):
    """Per-call latency of the drop-in API (api.py:120-186, 233-297; SURVEY §6 measured the reference's
    HilbertQuantizer.search of one query over 100 models at 21.2 ms in-container): quantize one 1024-d
    vector; search one query over 100 and over 10,000 registered models (the query's own quantize, JPEG and
    pre-computed index included, explicit candidate list); next to the reference-shaped port
    (oracle/hq_loops.py) doing the same per call on one host core."""
    import contextlib
    import io
    try:
        import PIL  # noqa: F401
    except ImportError:
        return {"skipped": "PIL not importable"}
    from hq_mi355x.api import HilbertQuantizer
    rng = np.random.default_rng(13)
    V = rng.standard_normal((10_100, 1024)).astype(np.float32)
    hq = HilbertQuantizer()
    res = {}
    with contextlib.redirect_stdout(io.StringIO()):
        hq.quantize(V[0], "warm")
        reps = 50
        t0 = time.perf_counter()
        for i in range(reps):
            hq.quantize(V[i], f"q{i}")
        res["quantize_ms"] = (time.perf_counter() - t0) / reps * 1e3
        models = hq.quantize_many(list(V[100:]), model_ids=[f"m{i}" for i in range(len(V) - 100)])
        queries = V[100:130] + 0.05 * rng.standard_normal((30, 1024)).astype(np.float32)
        for pool, name in ((models[:100], "search_100_ms"), (models, "search_10k_ms")):
            hq.search(queries[0], pool, 10)
            t0 = time.perf_counter()
            found = 0
            for q in queries:
                found += len(hq.search(q, pool, 10))
            res[name] = (time.perf_counter() - t0) / len(queries) * 1e3
            res[name.replace("_ms", "_results_per_call")] = found / len(queries)
    res["reference_search_100_ms_in_container"] = 21.2
    res["note"] = ("wall ms per call on the host thread (synchronous API: the query is quantized on the GPU, its "
                   "JPEG encoded on the host, the pool's resident corpus re-used while the candidate list holds the "
                   "same index arrays); SURVEY.md §6's 21.2 ms is the reference on the build container's CPU")
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_api(models, V, hq.compression_quality, args.cpu_seconds / 4)
    return res


def cpu_baseline_api(models, V, quality, seconds):
    """The reference's per-call work on one host core, reference-shaped (oracle/hq_loops.py): the query's
    quantize (per-element map + streaming tree + u8 normalise, PIL JPEG, per-square pre-computed index) and
    the candidate loop over 100 models' indices; the 10,000-model figure extrapolates the loop linearly."""
    from hq_mi355x.core.compressor import encode_jpeg
    from oracle import hq_loops as HL
    C = np.stack([m.hierarchical_indices for m in models[:100]])
    n, L = 32, C.shape[1]
    done, tq, ts, t0 = 0, 0.0, 0.0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        p = V[done % 30]
        a = time.perf_counter()
        encode_jpeg(HL.quantize_one(p, n, L), quality)
        HL.precomputed_one(p, n)
        b = time.perf_counter()
        from oracle import hq_oracle as O
        qidx = O.streaming_index(O.map_from_2d(O.map_to_2d(O.pad_parameters(p, n), n)), L)
        c = time.perf_counter()
        HL.progressive_search(qidx, C, 10, 0.1, 20)
        ts += time.perf_counter() - c
        tq += b - a
        done += 1
    return {"search_100_ms": (tq + ts) / done * 1e3, "search_10k_ms": (tq + 100 * ts) / done * 1e3,
            "quantize_ms": tq / done * 1e3, "unit": "ms per call", "cores": 1, "kind": "port",
            "sample": f"{done} calls: reference-shaped quantize (map, streaming tree, u8, PIL JPEG, per-square "
                      f"pre-computed index) + candidate loop over 100 models (oracle/hq_loops.py), single thread; "
                      f"10k = quantize + 100 x the 100-model loop"}


def main():
    args = parse()
    # multi-core CPU baseline first: worker processes are forked before anything initialises the GPU
    wr = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    cpu_par = cpu_baseline_parallel(args.dim, args.cpu_seconds / 4) if wr == (0, 1) and not args.no_cpu else None
    world, rank = dist_setup(args)
    from hq_mi355x import kernels as K
    if args.option:
        from hq_mi355x import _lib
        for o in args.option:
            name, value = o.split("=", 1)
            _lib.set_option(name, int(value))
    for o in args.py_set:  # host-side variants: module:attribute=int (A/B runs only)
        import importlib
        target, value = o.split("=", 1)
        mod, attr = target.split(":", 1)
        obj = importlib.import_module(mod)
        *path, attr = attr.split(".")  # module:Class.attribute too
        for a in path:
            obj = getattr(obj, a)
        old = getattr(obj, attr)
        setattr(obj, attr, value if isinstance(old, str) else type(old)(int(value)))
    from hq_mi355x.core.pipeline import quantize_batch

    dev = torch.device("cuda", torch.cuda.current_device())
    N, d = args.n_emb, args.dim
    n, L = 64, 64
    g = torch.Generator(device=dev).manual_seed(1 + 1000 * rank)
    X = torch.randn((N, d), generator=g, device=dev, dtype=torch.float32)
    frames = torch.empty((N, n + 1, n), dtype=torch.uint8, device=dev)
    idx = torch.empty((N, L), dtype=torch.float64, device=dev)
    mm = torch.empty((N, 2), dtype=torch.float32, device=dev)
    out = (frames, idx, mm)

    def step():
        quantize_batch(X, min_efficiency_ratio=0.2, index_space_size=L, out=out)

    wall, kern = timed(step, args.steps, args.warmup, world)
    ms = wall / args.steps * 1e3
    value = N * world * args.steps / wall
    bytes_per_emb = 4 * d + (n + 1) * n + 8 * L + 8
    achieved = bytes_per_emb * N / kern / 1e9
    traffic = load_traffic("k_fused_np64")
    rec = {
        "metric": "embeddings/sec Hilbert map+quantize (1536D)", "value": value, "unit": "embeddings/sec",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic N(0,1) float32 embeddings generated on device (seed 1 + 1000*rank)",
        "config": {"workload": "cfg2: 1M x 1536-d embeddings per GPU, order-64 Hilbert map + streaming index "
                               "(L=64, f64) + index-row embed + uint8 quantize (fused hq_map_index_quantize)",
                   "embeddings_per_gpu": N, "dim": d, "grid": n, "index_len": L,
                   "parallelism": f"dp{world} (independent shards, no collective)"},
        "roofline": hbm_roofline(achieved, traffic, algorithmic_bytes_per_embedding=bytes_per_emb,
                                 kernel_ms=kern * 1e3),
    }

    # the pre-computed index leg reads the headline's embeddings; run next to it, before the search legs
    # churn the allocator (measured: its kernel 4.01 ms here, 4.31 ms after the search legs)
    if not args.no_precomputed:
        rec["precomputed"] = bench_precomputed(args, X, world)

    if not args.no_search:
        from hq_mi355x.core.search_engine import IndexCorpus
        from hq_mi355x.distributed import ShardedIndexCorpus
        Nc, Qn = args.corpus, args.queries
        gc = torch.Generator(device=dev).manual_seed(2 + 1000 * rank)
        Xc = torch.randn((Nc, d), generator=gc, device=dev, dtype=torch.float32)
        _, corpus_idx, _ = K.map_index_quantize(Xc, n, L)
        del Xc
        # queries = global corpus rows 0..Q-1 (rank 0's shard) + N(0, 0.01) noise, identical on all ranks
        q0 = corpus_idx[:Qn].clone()
        if world > 1:
            import torch.distributed as dist
            dist.broadcast(q0, src=0)
        gq = torch.Generator(device=dev).manual_seed(3)
        queries = q0 + 0.01 * torch.randn(q0.shape, generator=gq, device=dev, dtype=torch.float64)
        torch.cuda.synchronize()
        tp0 = time.perf_counter()
        comm = None
        if world > 1:
            # the records all-gather runs through the C-ABI (hq_allgather_topk, RCCL over xGMI) when the
            # ranks hold one GPU each; the one-GPU rehearsal (HQ_BENCH_SAME_DEVICE + gloo) uses torch.distributed
            if os.environ.get("HQ_BENCH_BACKEND", "nccl") == "nccl":
                from hq_mi355x.rccl import Communicator
                comm = Communicator.from_process_group()
            engine = ShardedIndexCorpus(corpus_idx, id_base=rank * Nc, n_total=Nc * world, comm=comm)
        else:
            engine = IndexCorpus(corpus_idx)
        torch.cuda.synchronize()
        prep_s = time.perf_counter() - tp0
        # every step answers one whole 1000-query batch; batch i + 1 is queued before batch i's one host
        # sync (progressive_submit / progressive_finish), so the GPU does not idle on the host between
        # batches; the last batch is finished inside the timed region.  HQ_SEARCH_STREAMS=n (A/B knob)
        # alternates the batches over n HIP streams: 2 / 3 streams measured 1.43M / 0.7-1.05M vs 2.07M QPS
        # on one (two batches' scans contend for the CUs), so one stream is the default
        nstreams = int(os.environ.get("HQ_SEARCH_STREAMS", "1"))
        depth = SEARCH_DEPTH
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
        pend, nsub = [], [0]

        def run():
            st = streams[nsub[0] % len(streams)]
            nsub[0] += 1
            with torch.cuda.stream(st):
                pend.append((st, engine.progressive_submit(queries, 10, 0.1, 20)))
            if len(pend) >= depth:
                drain(1)

        def drain(n=None):
            while pend and (n is None or n > 0):
                st, p = pend.pop(0)
                with torch.cuda.stream(st):
                    engine.progressive_finish(p)
                n = None if n is None else n - 1

        swall, skern = timed(run, args.search_steps, 1, world, drain)
        qps = Qn * args.search_steps / swall
        pairs = Qn * Nc  # level-0 pairs scored per rank per step
        # the level-0 contraction once per pair (2 * 32 flops): the scan executes one f16 MFMA pass (hi.hi; the
        # split hi.lo + lo.hi terms only for the pre-filter's survivors, on the VALU), so the peak is the dense
        # f16 MFMA peak; rounds 1-3 counted the three split passes against it ("frac_split_accounting")
        flops = 2.0 * pairs * 32
        ids, ov, _, cnt = engine.progressive(queries, 10, 0.1, 20)
        rec["search"] = {
            "metric": "queries/sec@top-10 over 1M corpus", "value": qps, "unit": "queries/sec",
            "corpus_per_gpu": Nc, "corpus_total": Nc * world, "queries": Qn, "steps": args.search_steps,
            "ms_per_step": swall / args.search_steps * 1e3, "index_prepare_s": prep_s,
            "mode": "progressive (level-0 scan: hi.hi f16 MFMA pre-filter, split G of the survivors, top-28 >= 0.1 - "
                    f"eps; exact re-rank to top-20, overall re-score, top-10); up to {depth} batches in flight",
            "roofline": {"bound": "mfma", "achieved": flops / skern / 1e12, "peak": FP16_MATRIX_PEAK_TFS,
                         "unit": "TFLOP/s", "frac": flops / skern / 1e12 / FP16_MATRIX_PEAK_TFS,
                         "frac_split_accounting": 3 * flops / skern / 1e12 / FP16_MATRIX_PEAK_TFS,
                         "note": "2*Q*N*32 flops of the level-0 contraction per step (the one f16 MFMA pass the scan "
                                 "executes) / step time of the whole pipeline (sample pass, scan, pool select, exact "
                                 "re-rank, final); frac_split_accounting = rounds 1-3's count (three split passes)"},
            "self_match_rate": float((ids[:, 0].cpu() == torch.arange(Qn)).float().mean()),
        }
        # the other two cfg3 modes: brute-force overall top-10 (core/search_engine.py:302-338,
        # f64 MFMA scan over all segments + exact re-rank) and the video engine's strict level-0 frame scan
        # (core/video_search.py:215-264, split-f16 scan + exact re-rank, `>` threshold)
        # overall: the split-f16 contraction over every level value (K-blocks of 32: hq_seg_packov_info),
        # 3 MFMA passes (hi.hi, hi.lo, lo.hi) as the level-0 count; the f64 scan (no split layout) is
        # counted as 2*Q*N*Lp against the FP64 matrix peak
        ovinfo = K.packov_info(L)
        Lp = K.seg_padded_len(L)
        ov_flops, ov_peak, ov_pname = ((2.0 * pairs * 32 * ovinfo[0], FP16_MATRIX_PEAK_TFS, "dense F16 MFMA")
                                       if ovinfo else (2.0 * pairs * Lp, FP64_MATRIX_PEAK_TFS, "FP64 matrix (spec)"))
        modes = {}
        l0_flops = 2.0 * pairs * 32
        for mode, fn, flops, peak, pname in () if args.no_modes else (
                ("overall", lambda: engine.brute_force(queries, 10), ov_flops, ov_peak, ov_pname),
                ("level0", lambda: engine.frame_search(queries, 10, 0.1), l0_flops, FP16_MATRIX_PEAK_TFS,
                 "dense F16 MFMA"),
                # the reference engine's default max_candidates_per_level (core/search_engine.py:31,
                # core/video_search.py:48) and SearchConfig's (config.py:181): long pools on the scan path
                ("m100", lambda: engine.progressive(queries, 10, 0.1, 100), l0_flops, FP16_MATRIX_PEAK_TFS,
                 "dense F16 MFMA"),
                ("m1000", lambda: engine.progressive(queries, 10, 0.1, 1000), l0_flops, FP16_MATRIX_PEAK_TFS,
                 "dense F16 MFMA")):
            msteps = max(2, args.search_steps // 2)
            Mm = {"m100": 100, "m1000": 1000}.get(mode)
            sync = None
            if Mm is not None:
                # pipelined as the M = 20 leg (SEARCH_DEPTH batches in flight); the synchronous call's rate beside
                sw, _ = timed(fn, msteps, 1, world)
                sync = {"value": Qn * msteps / sw, "ms_per_step": sw / msteps * 1e3,
                        "note": "engine.progressive per step (submit + finish, the host waits for each batch)"}
                pend_m = []

                def fn(M=Mm):
                    pend_m.append(engine.progressive_submit(queries, 10, 0.1, M))
                    if len(pend_m) >= SEARCH_DEPTH:
                        engine.progressive_finish(pend_m.pop(0))

                def drain_m():
                    while pend_m:
                        engine.progressive_finish(pend_m.pop(0))
            mw, mk = timed(fn, msteps, 1, world, drain_m if Mm is not None else None)
            modes[mode] = {
                "value": Qn * msteps / mw, "unit": "queries/sec", "steps": msteps, "ms_per_step": mw / msteps * 1e3,
                "max_candidates_per_level": Mm, "pipelined": Mm is not None, "sync": sync,
                "roofline": {"bound": "mfma", "achieved": flops / mk / 1e12, "peak": peak, "unit": "TFLOP/s",
                             "frac": flops / mk / 1e12 / peak,
                             "note": f"contraction flops per step, one f16 pass ({('2*Q*N*32*K-blocks' if ovinfo else '2*Q*N*Lp f64') if mode == 'overall' else '2*Q*N*32'}) / "
                                     f"GPU step time (HIP events); peak = {pname}"}}
        rec["search"]["modes"] = modes
        if not args.no_hard and isinstance(engine, IndexCorpus):
            rec["search"]["modes"].update(bench_search_hard(args, engine, dev, n, L, world))
        if comm is not None:
            # the one collective of the sharded search alone: the records block of one batch per rank
            x = torch.zeros((Qn, 21, 3 + engine.local.nseg), dtype=torch.float64, device=dev)
            _, ak = timed(lambda: comm.all_gather(x), 20, 3, world)
            rec["search"]["allgather"] = {"ms": ak * 1e3, "bytes_per_rank": x.numel() * 8, "ranks": world,
                                          "path": "hq_allgather_topk (ncclAllGather over xGMI)"}
            comm.close()
        if args.corpus_total > 0:
            del engine
            torch.cuda.empty_cache()
            rec["search"]["strong"] = bench_search_strong(args, world, rank, dev)

    if not args.no_frames:
        rec["frames"] = bench_frames(args, world, rank, dev)

    if rank == 0 and world == 1 and not args.no_ingest:
        rec["ingest"] = bench_ingest(args)

    if rank == 0 and world == 1 and not args.no_api:
        rec["api"] = bench_api(args)

    if not args.no_stream:
        del X, frames, idx, mm, out
        rec["stream"] = bench_stream(args, world, rank, dev)

    if rank == 0 and world == 1 and not args.no_cpu:
        rec["cpu_baseline"] = cpu_baseline_quantize_loops(d, args.cpu_seconds / 2)
        rec["cpu_baseline"]["threads_available"] = os.cpu_count()
        rec["cpu_baseline"]["vectorised"] = cpu_baseline_quantize(d, args.cpu_seconds / 2)
        if cpu_par:
            v, w = cpu_par["quantize"]
            rec["cpu_baseline"]["multicore"] = {
                "value": v, "unit": "embeddings/sec", "cores": w, "kind": "port",
                "sample": f"NumPy oracle map+streaming index+embed+u8 normalise, 64-embedding batches, one process "
                          f"per core ({w} processes, {args.cpu_seconds / 4:.1f}s)"}
        if "search" in rec:
            from hq_mi355x._dev import to_np
            C = to_np(corpus_idx[:100_000])
            Qh = to_np(queries[:50])
            rec["search"]["cpu_baseline"] = cpu_baseline_search_loops(C, Qh, args.cpu_seconds / 2)
            rec["search"]["cpu_baseline"]["vectorised"] = cpu_baseline_search(C, Qh, args.cpu_seconds / 2)
            for mode in ("overall", "level0"):
                if mode in rec["search"].get("modes", {}):
                    rec["search"]["modes"][mode]["cpu_baseline"] = cpu_baseline_mode(mode, C, Qh, args.cpu_seconds / 4)
            if cpu_par:
                v, w = cpu_par["search"]
                rec["search"]["cpu_baseline"]["multicore"] = {
                    "value": v / 1_000_000, "unit": "queries/sec over a 1M corpus (extrapolated)", "cores": w,
                    "kind": "port", "sample": f"oracle progressive_search over a 20k-row corpus, one process per "
                                              f"core ({w} processes), linear in corpus size"}
        if "stream" in rec:
            rec["stream"]["cpu_baseline"] = cpu_baseline_stream(args.cpu_seconds / 2)
        if "precomputed" in rec:
            rec["precomputed"]["cpu_baseline"] = cpu_baseline_precomputed(d, args.cpu_seconds / 2)
    if rank == 0:
        rec["summary"] = summary(rec)  # last key: the end of the line a driver's short stdout tail keeps
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
