#!/bin/bash
# round-3 re-entry check: whole GPU suite + default bench at HEAD
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t9.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t9.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r03_b9.json 2> gpurun_out/r03_b9.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r03_b9.json; exit $rc
