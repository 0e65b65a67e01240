#!/bin/bash
# final ranking by arg-max rounds (default) against the sort only (final_rounds = 0): M = 100 / 1000 statistics
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_longlist.py -x -q --timeout 200 --timeout-method thread -k "fused_final or progressive_matches_oracle or sharded" > $O/r05_28_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r05_28_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do for m in m100 m1000; do
  cd /tmp && HQ_DBG_OPTS=final_rounds=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof28_${m}_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof28_${m}_$v.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  echo "final_rounds=$v $m: $(python3 tools/prof_summary.py $O/prof28_${m}_$v | grep -E 'k_rank_sort')"
done; done
