#!/bin/bash
# round-3 checkpoint 5 (rebuilt container): whole GPU suite, smoke, default bench, rocprof kernel stats of the bench
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_t32.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t32.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke32.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03_smoke32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r03_b32.json 2> gpurun_out/r03_b32.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b32 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > gpurun_out/prof_r03b32.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py gpurun_out/prof_r03b32 | head -20; exit $rc
