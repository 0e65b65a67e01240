#!/bin/bash
# S7 memory-phase order: 11 fragment reads before staging + loads, 12 global loads in the compute phase
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t29a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -2 gpurun_out/r03_t29a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_frames.sh - cos_kernel=11 cos_kernel=12 - cos_kernel=11 cos_kernel=12 > gpurun_out/r03_ab29.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab29.txt; exit $rc
