#!/bin/bash
# PMC passes of the cooperative long-list re-rank (k_rank_pairs) in the M = 1000 progressive search
export TMPDIR=/tmp
timeout -k 10 120 python tools/scan_debug.py m1000 > gpurun_out/rp_dry.log 2>&1 || { echo "dry run failed"; tail -5 gpurun_out/rp_dry.log; exit 1; }
bash tools/pmc_kernel.sh k_rank_pairs gpurun_out/pmc_rp m1000 > gpurun_out/pmc_rp.txt 2>&1 || { tail -5 gpurun_out/pmc_rp.txt; exit 1; }
cat gpurun_out/pmc_rp.txt
