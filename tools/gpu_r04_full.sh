#!/bin/bash
# round-4 checkpoint: whole GPU test suite, bench (N=1 default), rocprofv3 kernel statistics, smoke
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04_full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r04_full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r04_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/r04_bench_full.json 2> $O/r04_bench_full.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_r04full -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > $O/prof_r04full.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py $O/prof_r04full | head -30; exit $rc
