#!/bin/bash
# per-lane level tails in the cooperative re-rank: long-list + hard-query tests, statistics
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py -x -q --timeout 300 --timeout-method thread > $O/r05_20_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r05_20_tests.log; [ $rc -eq 0 ] || exit $rc
for m in m100 m1000; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof20_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof20_$m.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; echo "prof $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py $O/prof20_$m > $O/prof20_$m.txt; grep -E "scan0g|rank_|pool_s|final|sample_topg" $O/prof20_$m.txt
done
