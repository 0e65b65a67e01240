#!/bin/bash
# tiled-layout cosine kernel v2 (branch-free pipeline): parity, A/B FT = 2 / 1 / 4 vs the ping-pong kernel
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t11a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -3 gpurun_out/r03_t11a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab_frames.sh - cos_kernel=4 cos_kernel=5 cos_kernel=3 - > gpurun_out/r03_ab11.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab11.txt; exit $rc
