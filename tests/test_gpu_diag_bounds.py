"""Bounds guard: the level-0 scan's corpus-row loads run once through the DIAG library
(`make DIAG=1`: every guarded load checks its row against the padded copies and counts violations instead
of faulting) on the corpus shapes of the round-2 fault class (chunks past N, ragged chunk ends, N not a
multiple of 4), and the default library gives the same results."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_LIB = os.path.join(ROOT, "hilbert-quantization_amd", "hq_mi355x", "libhq_mi355x_diag.so")


@pytest.mark.gpu
def test_level0_scan_rows_in_bounds_diag_build(hq_lib, tmp_path):
    if not os.path.exists(DIAG_LIB):
        pytest.fail(f"{DIAG_LIB} missing: build it with `make -C hilbert-quantization_amd/csrc DIAG=1` "
                    "(__graft_entry__.build() does)")
    worker = os.path.join(ROOT, "tests", "diag_bounds_worker.py")
    out = {}
    for tag, env in (("diag", {"HQ_LIB_VARIANT": DIAG_LIB}), ("release", {})):
        path = str(tmp_path / f"{tag}.npz")
        e = dict(os.environ)
        e.pop("HQ_LIB_VARIANT", None)
        e.update(env)
        r = subprocess.run([sys.executable, "-u", worker, path], env=e, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        with np.load(path) as z:
            out[tag] = {k: z[k] for k in z.files}
    d, rel = out["diag"], out["release"]
    assert int(d["diag"]) == 1 and int(rel["diag"]) == 0
    assert int(d["violations"]) == 0, f"{int(d['violations'])} out-of-bounds rows, first at hq_search.hip:{int(d['line'])}"
    for k in d:
        if k[0] in "pf":
            np.testing.assert_array_equal(d[k], rel[k], err_msg=k)
