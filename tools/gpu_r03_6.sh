#!/bin/bash
# overall split scan: new parity test, search tests, then the overall mode in the bench under rocprof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t6.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t6.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_scan.sh default
python3 tools/prof_summary.py gpurun_out/ab_1 | head -24
grep -o '"overall": {[^}]*' gpurun_out/ab_1.log | head -c 300; echo
