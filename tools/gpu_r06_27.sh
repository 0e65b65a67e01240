#!/bin/bash
# k_pool_sort: wave-aggregated radix histogram (option pool_agg): parity, A/B, kernel times
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_longlist.py > $O/r06_27_tests.log 2>&1 || { tail -30 $O/r06_27_tests.log; exit 1; }
tail -2 $O/r06_27_tests.log
for w in 0 1; do
  cd /tmp && HQ_DBG_OPTS=pool_agg=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r06_27_a${w} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py m1000 > $O/r06_27_a${w}.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT; echo "pool_agg=$w m1000"; python3 tools/prof_summary.py $O/r06_27_a${w} | grep -E "k_pool_sort" | head -3
done
bash tools/ab_bench_search.sh r06_27_ab "agg0|" "agg1|--option pool_agg=1" || exit 1
