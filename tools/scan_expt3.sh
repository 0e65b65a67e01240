#!/bin/bash
# contiguous-load experiment (HQ_SCAN_EXPT=10) across waves per block / prefetch distance
export TMPDIR=/tmp
export HQ_LIB_VARIANT=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for c in "1 2" "4 2" "1 3" "4 3" "1 4"; do
  set -- $c
  HQ_SCAN_EXPT=10 HQ_SCAN_WPB=$1 HQ_SCAN_PF=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sz_$1_$2 -o run --output-format csv -- python3 tools/scan_debug.py > gpurun_out/sz_$1_$2.log 2>&1 || { echo "$c failed"; tail -3 gpurun_out/sz_$1_$2.log; exit 1; }
  echo "wpb $1 pf $2: $(python3 tools/prof_summary.py gpurun_out/sz_$1_$2 | grep -E 'k_scan0g' | tr -s ' ' | cut -c1-120)"
done
