#!/bin/bash
# level-0 scan at 3 waves per SIMD with a deeper prefetch (options scan_occ 3, scan_pf 6 / 8), the K'-th
# bisection's query statistics prefetched, the register-resident level-0 bitonic (option rank_sort_reg):
# parity, A/B, kernel statistics
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_longlist.py -x -q --timeout 300 --timeout-method thread > $O/r06_11_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_11_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench_search.sh r06_11_ab "default|" "rank_sort_reg=0|--option rank_sort_reg=0" "scan_occ=3 pf6|--option scan_occ=3 --option scan_pf=6" "scan_occ=3 pf8|--option scan_occ=3 --option scan_pf=8" || exit 1
for v in "" "rank_sort_reg=0" "scan_occ=3,scan_pf=8"; do for m in m20 m100 m1000; do
  cd /tmp && HQ_DBG_OPTS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof11_${m}_${v:-def} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof11_${m}.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "${v:-default} $m: $(python3 tools/prof_summary.py $O/prof11_${m}_${v:-def} | grep -E 'scan0g|sample_kth|rank_sort' | tr -s ' ' | cut -c1-100 | tr '\n' ';')"
done; done
