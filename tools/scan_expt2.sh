#!/bin/bash
# level-0 scan timing experiments (diagnostics build): 0 normal, 6 nothing queued, 7 no pre-filter,
# 9 no fragment loads in the loop
export TMPDIR=/tmp
export HQ_LIB_VARIANT=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for e in ${EXPTS:-0 7 10}; do
  HQ_SCAN_EXPT=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sy_${e} -o run --output-format csv -- python3 tools/scan_debug.py > gpurun_out/sy_${e}.log 2>&1 || { echo "expt $e failed"; tail -3 gpurun_out/sy_${e}.log; exit 1; }
  echo "expt $e: $(python3 tools/prof_summary.py gpurun_out/sy_${e} | grep -E 'k_scan0g' | tr -s ' ' | cut -c1-120)"
done
