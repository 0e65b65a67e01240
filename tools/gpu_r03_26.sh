#!/bin/bash
# S7: L2 touch-ahead of the frame fragments (cos_kernel 9: 4 steps, 10: 8 steps) — parity + A/B
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t26a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -2 gpurun_out/r03_t26a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_frames.sh - cos_kernel=9 cos_kernel=10 - cos_kernel=9 cos_kernel=10 > gpurun_out/r03_ab26.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab26.txt; exit $rc
