#!/bin/bash
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 200 python tools/pool_sizes.py > $O/r05_13.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r05_13.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests/test_gpu_hard_queries.py -x -v -s --timeout 600 --timeout-method thread --durations=0 > $O/r05_12_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "M=|passed|failed|Error|s call" $O/r05_12_tests.log | head -20; exit $rc
