#!/bin/bash
# round 5, call 2: cooperative vs per-thread long-list re-rank timing (+ kernel trace); hard query tests
# with the longer-list retry; trimmed bench
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/refine_timing.py > $O/r05_2_refine.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r05_2_refine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_hard_queries.py -x -v -s --timeout 600 --timeout-method thread --durations=0 > $O/r05_2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "M=|passed|failed|Error" $O/r05_2_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-stream --no-precomputed --no-ingest --no-frames --no-api --corpus-total 0 \
  --search-steps 10 --no-cpu > $O/r05_2_bench.json 2> $O/r05_2_bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r05_2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/refine_timing.py > $O/r05_2_prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; python3 tools/prof_summary.py $O/prof_r05_2; exit $rc
