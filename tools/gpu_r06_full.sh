#!/bin/bash
# round-6 checkpoint: whole GPU test suite, smoke, default bench (N=1), rocprofv3 kernel statistics of the bench
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
V=${1:-v1}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06_full_tests_$V.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r06_full_tests_$V.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r06_smoke_$V.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r06_smoke_$V.log; [ $rc -eq 0 ] || exit $rc
T0=$(date +%s); timeout -k 10 500 python bench.py > $O/r06_bench_$V.json 2> $O/r06_bench_$V.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - T0 ))s"; [ $rc -eq 0 ] || exit $rc
[ "$2" = "noprof" ] && exit 0
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_r06_$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu > $O/prof_r06_$V.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo "prof rc=$rc"; python3 tools/prof_summary.py $O/prof_r06_$V | head -24; exit $rc
