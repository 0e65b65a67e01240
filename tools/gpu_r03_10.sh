#!/bin/bash
# tiled-layout cosine kernel: parity, A/B against the LDS-DMA ping-pong kernel, then the whole suite + bench
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t10a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -3 gpurun_out/r03_t10a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab_frames.sh - cos_kernel=3 - cos_kernel=3 > gpurun_out/r03_ab10.txt 2>&1
rc=$?; cat gpurun_out/r03_ab10.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t10.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t10.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r03_b10.json 2> gpurun_out/r03_b10.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r03_b10.json; exit $rc
