#!/bin/bash
# level-0 scan timing experiments on the diagnostics build: expt 0 (normal), 5 (fragments of step 0 only:
# no memory latency), 6 (5 + nothing queued), each at 1 and 4 waves per block
export TMPDIR=/tmp
export HQ_LIB_VARIANT=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for e in 0 5 6; do
  for w in 1 4; do
    HQ_SCAN_EXPT=$e HQ_SCAN_WPB=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sx_${e}_$w -o run --output-format csv -- python3 tools/scan_debug.py > gpurun_out/sx_${e}_$w.log 2>&1 || { echo "expt $e $w failed"; tail -3 gpurun_out/sx_${e}_$w.log; exit 1; }
    echo "expt $e wpb $w: $(python3 tools/prof_summary.py gpurun_out/sx_${e}_$w | grep -E 'k_scan0g|k_sample_topf' | tr -s ' ' | cut -c1-120 | tr '\n' ';')"
  done
done
