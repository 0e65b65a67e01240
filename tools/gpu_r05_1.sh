#!/bin/bash
# round 5, call 1: cooperative long-list re-rank parity; hard query distributions (fresh / clustered) at
# full size vs the dense exact path; trimmed bench (headline + search + hard modes + api)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_longlist.py -x -v --timeout 300 --timeout-method thread > $O/r05_1_longlist.log 2>&1
rc=$?; echo "longlist rc=$rc"; tail -5 $O/r05_1_longlist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-stream --no-precomputed --no-ingest --no-frames --corpus-total 0 \
  --search-steps 10 --cpu-seconds 8 > $O/r05_1_bench.json 2> $O/r05_1_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 $O/r05_1_bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_hard_queries.py -x -v --timeout 600 --timeout-method thread --durations=0 > $O/r05_1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $O/r05_1_tests.log; exit $rc
