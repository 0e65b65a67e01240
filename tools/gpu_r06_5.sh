#!/bin/bash
# compile-time level structures in the cooperative scorers (option rank_ct) and one ballot per block of rows in
# k_scanov (option ov_any): parity, A/B, kernel statistics, PMC; the clustered corpus's cold first batch
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py -x -q --timeout 300 --timeout-method thread > $O/r06_5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ov_check.py > $O/r06_5_ovcheck.log 2>&1; rc=$?; echo "ov_check rc=$rc"; grep -v amdgpu.ids $O/r06_5_ovcheck.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench_search.sh r06_5_ab "default (rank_ct=1, ov_any=1)|" "rank_ct=0|--option rank_ct=0" "rank_ct=2|--option rank_ct=2" "ov_any=0|--option ov_any=0" || exit 1
for v in 0 1; do for m in m20 m100 m1000; do
  cd /tmp && HQ_DBG_OPTS=rank_ct=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof5_${m}_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof5_${m}_$v.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "rank_ct=$v $m: $(python3 tools/prof_summary.py $O/prof5_${m}_$v | grep -E 'k_rank_pairs|k_rank_small' | head -1 | tr -s ' ' | cut -c1-150)"
done; done
for v in 1 0; do
  cd /tmp && HQ_DBG_OPTS=ov_any=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof5_ov_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py overall > $O/prof5_ov_$v.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
  echo "ov_any=$v: $(python3 tools/prof_summary.py $O/prof5_ov_$v | grep -E 'k_scanov<' | head -1 | tr -s ' ' | cut -c1-160)"
done
timeout -k 10 300 python tools/cold_batch_prof.py > $O/r06_5_cold.log 2>&1; echo "cold rc=$?"; grep -E "batch:" $O/r06_5_cold.log
timeout -k 10 300 bash tools/pmc_kernel.sh "k_scanov<" $O/r06_5_pmc_scanov overall > $O/r06_5_pmc_scanov.txt 2>&1; echo "pmc scanov rc=$?"; tail -3 $O/r06_5_pmc_scanov.txt
timeout -k 10 300 bash tools/pmc_kernel.sh k_sample_topg $O/r06_5_pmc_sample level0 > $O/r06_5_pmc_sample.txt 2>&1; echo "pmc sample rc=$?"; tail -3 $O/r06_5_pmc_sample.txt
