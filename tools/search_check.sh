#!/bin/bash
# Search parity tests + a search-only bench line + a kernel trace of it.  usage: tools/search_check.sh <tag>
set -u
TAG=${1:-s}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_search.py tests/test_gpu_search_f32.py -m gpu > $OUT/search_tests_$TAG.log 2>&1; rc=$?
tail -3 $OUT/search_tests_$TAG.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
for v in ${VARIANTS:-0}; do
  HQ_SCAN0_V=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 > $OUT/search_bench_${TAG}_v$v.json 2> $OUT/search_bench_${TAG}_v$v.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $OUT/search_bench_${TAG}_v$v.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/search_bench_${TAG}_v$v.json'));s=d['search'];print('V=$v QPS',round(s['value']),'ms',s['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sprof_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 10 > $OUT/sprof_$TAG.log 2>&1
f=$(find $OUT/sprof_$TAG -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-4
