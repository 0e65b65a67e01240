#!/bin/bash
# k_rank_sort<128, 128> for lists <= 128 (option rank_sort_small): parity, A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py > $O/r06_25_tests.log 2>&1 || { tail -30 $O/r06_25_tests.log; exit 1; }
tail -3 $O/r06_25_tests.log
bash tools/ab_bench_search.sh r06_25_ab "small|" "no small|--option rank_sort_small=0" || exit 1
