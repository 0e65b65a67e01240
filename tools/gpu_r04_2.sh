#!/bin/bash
# (1) round-3 head baseline (.baseline/: git archive of the round-3 head + its library): bench + kernel trace
# (2) this tree: the GPU suite (long lists, API goldens, hi.hi scan), smoke, bench
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
( cd .baseline && timeout -k 10 400 python bench.py > $O/r04_b1.json 2> $O/r04_b1.err ); rc=$?; echo "base bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
( cd .baseline && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_r04b1 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > $O/prof_r04b1.log 2>&1 ); rc=$?; echo "base prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04_t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/r04_t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > $O/r04_b2.json 2> $O/r04_b2.err; rc=$?; echo "bench rc=$rc"; exit $rc
