#!/bin/bash
# k_rank_sort with 256 threads for lists > 512 (option rank_sort_nt 256): parity, A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_longlist.py -k "window or cooperative or fused_final" > $O/r06_24_tests.log 2>&1 || { tail -30 $O/r06_24_tests.log; exit 1; }
tail -3 $O/r06_24_tests.log
bash tools/ab_bench_search.sh r06_24_ab "nt512|" "nt256|--option rank_sort_nt=256" || exit 1
