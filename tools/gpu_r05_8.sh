#!/bin/bash
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py -x -q --timeout 300 --timeout-method thread > $O/r05_8_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r05_8_tests.log; exit $rc
