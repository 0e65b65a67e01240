#!/bin/bash
# k_cos_t epilogue: parity (incl. wide stores), A/B FT3/D1 8-byte vs 16-byte stores, no-store diagnostic
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x -k cosine --timeout 120 --timeout-method thread > gpurun_out/r03_t13a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -3 gpurun_out/r03_t13a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab_frames.sh cos_kernel=6 cos_kernel=8 - cos_kernel=6 cos_kernel=8 > gpurun_out/r03_ab13.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03_ab13.txt; [ $rc -eq 0 ] || exit $rc
HQ_LIB_VARIANT=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so HQ_COS_KERNEL=90 timeout -k 10 120 python bench.py --no-search --no-stream --no-precomputed --no-ingest --no-cpu --steps 2 > gpurun_out/r03_ab13_ns.json 2>/dev/null
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r03_ab13_ns.json'))['frames']; print('no-store diag', round(d['value']/1e9,2), round(d['roofline']['frac'],3), round(d['ms_per_step'],3))"; exit $rc
