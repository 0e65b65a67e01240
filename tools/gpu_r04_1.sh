#!/bin/bash
# Round-4 baseline on the unchanged round-3 head: GPU suite, smoke, default bench, kernel trace
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke1.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r04_smoke1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r04_b1.json 2> gpurun_out/r04_b1.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04b1 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > gpurun_out/prof_r04b1.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py gpurun_out/prof_r04b1 | head -20; exit $rc
