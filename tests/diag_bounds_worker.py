"""Worker of tests/test_gpu_diag_bounds.py: runs level-0 scans through the DIAG library (bounds-guarded
corpus-row loads, hq_diag_violations) on the corpus shapes of the round-2 fault class and writes the
results and the violation count to an .npz.  Run as a child process with HQ_LIB_VARIANT set."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]

SHAPES = [(1, 5), (17, 5), (3000, 5), (3001, 64), (3056, 65), (4096, 1), (10_007, 130), (70_000, 1000)]


def main(out_path):
    import torch
    from hq_mi355x import _lib
    from hq_mi355x._dev import to_np
    from hq_mi355x.core.search_engine import IndexCorpus
    lib = _lib.lib()
    res = {"diag": np.array(lib.hq_diag_build())}
    for N, Q in SHAPES:
        rng = np.random.default_rng(N + Q)
        C = rng.standard_normal((N, 64))
        q = C[rng.integers(0, N, Q)] + rng.normal(0, 0.01, (Q, 64))
        corpus = IndexCorpus(C)
        ids, ov, _, cnt = corpus.progressive(q, 10, 0.1, 20)
        fids, fsc = corpus.frame_search(q, 10, 0.1)
        res[f"p{N}_{Q}"] = to_np(ids)
        res[f"f{N}_{Q}"] = to_np(fids)
    torch.cuda.synchronize()
    cnt, line = ctypes.c_int64(0), ctypes.c_int(0)
    _lib.check(lib.hq_diag_violations(ctypes.byref(cnt), ctypes.byref(line)))
    res["violations"] = np.array(cnt.value)
    res["line"] = np.array(line.value)
    np.savez(out_path, **res)


if __name__ == "__main__":
    main(sys.argv[1])
