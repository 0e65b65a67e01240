#!/bin/bash
# k_scanov PMC: LIN bound (default) vs the med3 + fma bound (scanov_v1)
export TMPDIR=/tmp
bash tools/pmc_kernel.sh k_scanov gpurun_out/pmc_ov_lin overall > gpurun_out/pmc_ov_lin.txt 2>&1 || { tail -5 gpurun_out/pmc_ov_lin.txt; exit 1; }
HQ_DBG_OPTS=scanov_v1=1 bash tools/pmc_kernel.sh k_scanov gpurun_out/pmc_ov_v1 overall > gpurun_out/pmc_ov_v1.txt 2>&1 || { tail -5 gpurun_out/pmc_ov_v1.txt; exit 1; }
cat gpurun_out/pmc_ov_lin.txt gpurun_out/pmc_ov_v1.txt
