#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t21a.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -2 gpurun_out/r03_t21a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/search_submit_time.py 2>&1 | tail -3
