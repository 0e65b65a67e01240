#!/bin/bash
# PMC passes of k_pool_sort at M = 1000
export TMPDIR=/tmp
bash tools/pmc_kernel.sh k_pool_sort gpurun_out/pmc_r06_pool_sort m1000 > gpurun_out/pmc_r06_pool_sort.txt 2>&1 || { tail -5 gpurun_out/pmc_r06_pool_sort.txt; exit 1; }
cat gpurun_out/pmc_r06_pool_sort.txt
