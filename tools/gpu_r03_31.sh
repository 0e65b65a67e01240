#!/bin/bash
# two-process sharded search on one GPU (gloo), then the CPU-side distributed tests for comparison
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t31.log 2>&1
rc=$?; echo "dist tests rc=$rc"; tail -30 gpurun_out/r03_t31.log; exit $rc
