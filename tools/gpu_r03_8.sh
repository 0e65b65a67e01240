#!/bin/bash
# round-3 checkpoint: whole GPU suite, default bench, rocprof kernel stats of the bench, PMC of k_scan0g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_t8.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py > gpurun_out/r03_b8.json 2> gpurun_out/r03_b8.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b8 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > gpurun_out/prof_r03b8.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_kernel.sh k_scan0g gpurun_out/pmc_scan0g_r03 level0 > gpurun_out/pmc_scan0g_r03.txt 2>&1; echo "pmc rc=$?"
