#!/bin/bash
# flagged-row pass folded into k_pool_select (k_scan0_flagged launch removed): whole GPU suite, DIAG bounds
# test included, then the default bench and its kernel trace
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_t33.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t33.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke33.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03_smoke33.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r03_b33.json 2> gpurun_out/r03_b33.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b33 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > gpurun_out/prof_r03b33.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py gpurun_out/prof_r03b33 | head -20; exit $rc
