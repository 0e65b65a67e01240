#!/bin/bash
# fused final ranking without the level-0 lists (selection rounds instead of the level-0 sort): parity, A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > $O/r06_10_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_10_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench_search.sh r06_10_ab "no level-0 lists (default)|" "level-0 lists + sort|--py-set hq_mi355x.kernels:FINAL_LEVEL0_LISTS=1" "ov_occ=3|--option ov_occ=3" "ov_occ=3 ov_any=1|--option ov_occ=3 --option ov_any=1" || exit 1
for m in m100 m1000; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof10_${m} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof10_${m}.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "$m: $(python3 tools/prof_summary.py $O/prof10_${m} | grep -E 'k_rank_pairs|k_rank_sort|pool_sort|scan0g' | tr -s ' ' | cut -c1-100 | tr '\n' ';')"
done
