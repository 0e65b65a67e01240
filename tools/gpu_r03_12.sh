#!/bin/bash
# k_cos_t variants: parity, A/B (FT = 3 / prefetch distance 1), PMC passes of the default
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t12a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -3 gpurun_out/r03_t12a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab_frames.sh - cos_kernel=6 cos_kernel=7 - cos_kernel=6 > gpurun_out/r03_ab12.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab12.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/pmc_cos.sh cos_t > gpurun_out/r03_pmc12.txt 2>&1; rc=$?; tail -30 gpurun_out/r03_pmc12.txt; exit $rc
