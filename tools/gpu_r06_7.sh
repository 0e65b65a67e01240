#!/bin/bash
# the re-rank's staging in one round trip (rank_stage) and k_pool_select's first loads together: parity, A/B
# against the previous library (variants/libhq_base_v2.so), kernel statistics
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py tests/test_gpu_threads.py tests/test_gpu_hard_queries.py -x -q --timeout 300 --timeout-method thread > $O/r06_7_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_7_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench_search.sh r06_7_ab "new|" "base (v2)||$GRAFT_REPO_ROOT/variants/libhq_base_v2.so" || exit 1
for m in m20 m100 m1000; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof7_${m} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof7_${m}.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "$m: $(python3 tools/prof_summary.py $O/prof7_${m} | grep -E 'k_rank_pairs|k_rank_small|pool_select|pool_sort' | tr -s ' ' | cut -c1-110 | tr '\n' ';')"
done
