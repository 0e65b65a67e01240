#!/bin/bash
# Round-4 baseline: the round-3 head (git archive HEAD + its built library in .baseline/): GPU suite, smoke,
# default bench, kernel trace.  Outputs under the top-level gpurun_out/.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd .baseline || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/r04_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r04_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke1.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r04_smoke1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/r04_b1.json 2> $O/r04_b1.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_r04b1 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > $O/prof_r04b1.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py $O/prof_r04b1 | head -20; exit $rc
