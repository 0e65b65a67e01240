#!/bin/bash
# fresh PMC passes: k_rank_pairs at M = 1000 and k_scanov (overall scan)
export TMPDIR=/tmp
bash tools/pmc_kernel.sh k_rank_pairs gpurun_out/pmc_r06_rank_pairs m1000 > gpurun_out/pmc_r06_rank_pairs.txt 2>&1 || { tail -5 gpurun_out/pmc_r06_rank_pairs.txt; exit 1; }
cat gpurun_out/pmc_r06_rank_pairs.txt
bash tools/pmc_kernel.sh k_scanov gpurun_out/pmc_r06_scanov overall > gpurun_out/pmc_r06_scanov.txt 2>&1 || { tail -5 gpurun_out/pmc_r06_scanov.txt; exit 1; }
cat gpurun_out/pmc_r06_scanov.txt
