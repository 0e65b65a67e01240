#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Stops at the first fault/timeout.
# usage: tools/gpu_check.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # pytest: 0 pass, 1 test failures (no fault)
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > $OUT/gpu_tests_$TAG.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests_$TAG.log
ok $rc || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 600 python bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
cat $OUT/bench_$TAG.json; tail -3 $OUT/bench_$TAG.err
[ $rc -eq 0 ] || { echo "bench rc=$rc: stopping"; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --no-ingest > $OUT/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"
find $OUT/prof_$TAG -name "*stats*" | head
exit 0
