#!/bin/bash
# PMC passes of the long-list re-rank (k_refine_big_sm_raw) in the M = 1000 progressive search
export TMPDIR=/tmp
timeout -k 10 60 python tools/scan_debug.py m1000 > gpurun_out/rf_dry.log 2>&1 || { echo "dry run failed"; tail -5 gpurun_out/rf_dry.log; exit 1; }
bash tools/pmc_kernel.sh k_refine_big_sm_raw gpurun_out/pmc_rf m1000 > gpurun_out/pmc_rf.txt 2>&1 || { tail -5 gpurun_out/pmc_rf.txt; exit 1; }
cat gpurun_out/pmc_rf.txt
