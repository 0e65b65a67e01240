#!/bin/bash
# radix-select k_pool_sort: long-list tests, hard-query tests, per-M kernel statistics
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py tests/test_gpu_search.py -x -q --timeout 300 --timeout-method thread > $O/r05_14_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r05_14_tests.log; [ $rc -eq 0 ] || exit $rc
for m in m100 m1000; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof14_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof14_$m.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; echo "prof $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py $O/prof14_$m | head -14
done
