#!/bin/bash
# search step timeline (kernel trace, gaps) + PMC traffic of the default k_cos_t
export TMPDIR=/tmp
bash tools/search_only_prof.sh r03t > gpurun_out/r03_sprof.txt 2>&1; rc=$?; cat gpurun_out/r03_sprof.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_gaps.py gpurun_out/sprof_r03t k_sample_topg 10 > gpurun_out/r03_gaps.txt 2>&1; cat gpurun_out/r03_gaps.txt
timeout -k 10 500 bash tools/pmc_cos.sh cos_t3 > gpurun_out/r03_pmc14.txt 2>&1; rc=$?; tail -3 gpurun_out/r03_pmc14.txt; exit $rc
