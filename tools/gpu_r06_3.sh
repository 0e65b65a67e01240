#!/bin/bash
# compile-time level structures in the cooperative scorers (option rank_ct): parity, A/B, kernel statistics;
# the clustered corpus's cold first batch under cProfile
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py -x -q --timeout 300 --timeout-method thread > $O/r06_3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_3_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench_search.sh r06_3_ab "rank_ct=1 (default)|" "rank_ct=0|--option rank_ct=0" "rank_ct=2|--option rank_ct=2" || exit 1
for v in 0 1 2; do for m in m20 m100 m1000; do
  cd /tmp && HQ_DBG_OPTS=rank_ct=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof3_${m}_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof3_${m}_$v.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "rank_ct=$v $m: $(python3 tools/prof_summary.py $O/prof3_${m}_$v | grep -E 'k_rank_pairs|k_rank_small' | head -2 | tr -s ' ' | cut -c1-150)"
done; done
timeout -k 10 300 python tools/cold_batch_prof.py > $O/r06_3_cold.log 2>&1; echo "cold rc=$?"; grep -E "batch:" $O/r06_3_cold.log
