#!/bin/bash
# overall scan: search tests, the search leg under rocprof, then PMC passes of k_scanov
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t7.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t7.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_scan.sh default || exit 1
python3 tools/prof_summary.py gpurun_out/ab_1 | grep -E "scanov|sampleov|scan0g"
grep -o '"overall": {[^}]*' gpurun_out/ab_1.log | head -c 200; echo
bash tools/pmc_kernel.sh k_scanov gpurun_out/pmc_scanov overall > gpurun_out/pmc_scanov.txt 2>&1; rc=$?; cat gpurun_out/pmc_scanov.txt; exit $rc
