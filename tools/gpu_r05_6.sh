#!/bin/bash
# round 5, call 6: sort-based dense select (k > 64) parity + the search legs
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py -x -q --timeout 300 --timeout-method thread > $O/r05_6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r05_6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --no-stream --no-precomputed --no-ingest --no-frames --no-api --corpus-total 0 \
  --no-cpu > $O/r05_6_bench.json 2> $O/r05_6_bench.err; rc=$?; echo "bench rc=$rc"; exit $rc
