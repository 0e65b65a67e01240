#!/bin/bash
# this tree: the GPU suite (long lists, API goldens, sort keys, hi.hi scans), smoke, bench (no CPU legs), kernel trace
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r04_t3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 $O/r04_t3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu > $O/r04_b3.json 2> $O/r04_b3.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_r04b3 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > $O/prof_r04b3.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py $O/prof_r04b3 | head -24; exit $rc
