#!/bin/bash
# PMC passes of k_rank_sort at M = 1000 (window ranking) and the kernel times by option rank_win
export TMPDIR=/tmp
bash tools/pmc_kernel.sh k_rank_sort gpurun_out/pmc_r06_rank_sort m1000 > gpurun_out/pmc_r06_rank_sort.txt 2>&1 || { tail -5 gpurun_out/pmc_r06_rank_sort.txt; exit 1; }
cat gpurun_out/pmc_r06_rank_sort.txt
