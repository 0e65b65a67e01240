#!/bin/bash
# exact re-rank / re-score reading only the candidates' raw rows: parity tests, then timing
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_search_f32.py tests/test_gpu_api_golden.py tests/test_gpu_sortkey.py -q -x --timeout 300 --timeout-method thread > $O/rt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/rt_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/refine_timing.py
