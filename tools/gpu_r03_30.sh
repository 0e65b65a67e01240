#!/bin/bash
# S7 wide query tile k_cos_w (cos_kernel 13: 256 queries x 256 frames, query fragments read in the compute phase)
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_fullsize.py -q -x -k "cosine or frames" --timeout 200 --timeout-method thread > gpurun_out/r03_t30a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -2 gpurun_out/r03_t30a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_frames.sh - cos_kernel=13 - cos_kernel=13 > gpurun_out/r03_ab30.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab30.txt; exit $rc
