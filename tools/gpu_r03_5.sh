#!/bin/bash
# search tests, then A/B of the sample pass variants
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py tests/test_gpu_fullsize.py tests/test_gpu_diag_bounds.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t5.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t5.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_scan.sh "$@"
