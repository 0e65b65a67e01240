#!/bin/bash
# round 6: re-entrancy (8-thread) tests, the sharded retry test, and the search suites they touch
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_hard_queries.py tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_distributed.py -x -v -s --durations=15 --timeout 300 --timeout-method thread > $O/r06_1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 $O/r06_1_tests.log; exit $rc
