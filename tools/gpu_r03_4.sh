#!/bin/bash
# full GPU suite, then the search leg (default scan and the list-based scan_variant=1) under rocprof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t4.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r03_t4.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_scan.sh default scan_variant=1
