#!/bin/bash
# k_rank_sort window ranking (option rank_win): parity tests, then A/B against the sort alone
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py > $O/r06_21_tests.log 2>&1 || { tail -30 $O/r06_21_tests.log; exit 1; }
tail -3 $O/r06_21_tests.log
bash tools/ab_bench_search.sh r06_21_ab "rank_win=1 (window)|" "rank_win=0 (sort)|--option rank_win=0" || exit 1
