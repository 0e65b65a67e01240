"""The sharded search in real processes on the GPU: two ranks (torch.distributed.run,
both on cuda:0, gloo for the records all-gather) each hold a contiguous shard in a ShardedIndexCorpus;
the merged progressive, brute-force and frame-scan results (hq_progressive_final / the R-way merges)
equal the unsharded IndexCorpus bit for bit, and sampled queries equal the oracle
(core/search_engine.py:232-388; merge analogue core/video_search.py:722-875).  The CPU rehearsal of the
protocol is tests/test_distributed_cpu.py; the 8-shard cfg4 merge is in tests/test_gpu_fullsize.py."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.parametrize("backend", ["gloo", "rccl"])
def test_sharded_search_two_processes(hq_lib, backend):
    """gloo: both ranks on cuda:0 (runs on a one-GPU box); rccl: one GPU per rank with the records
    all-gather through the C-ABI (hq_allgather_topk) — runs where two GPUs are visible."""
    if backend == "rccl" and _device_count() < 2:
        pytest.skip("the RCCL form needs two GPUs (one rank per GPU)")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        if backend == "rccl":
            env["HQ_DIST_RCCL"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "_dist_gpu_worker.py"), out]
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        res = json.load(open(out + ".json"))
        assert res["world"] == 2
        for mode, eq in res["equal"].items():
            assert all(eq), (mode, eq)
        z = np.load(out + ".npz")
        C, Q, ids, ov, cnt = z["C"], z["Q"], z["ids"], z["ov"], z["cnt"]
        for a in (0, 1, 2, 3, 30, 66):
            rid, rsc, _, _ = O.progressive_search(Q[a], C, 10, 0.1, 20)
            assert list(ids[a][: cnt[a]]) == list(rid), a
            np.testing.assert_allclose(ov[a][: cnt[a]], rsc, atol=1e-10)
