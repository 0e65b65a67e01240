#!/bin/bash
# search tests + search-leg kernel profiles: default scan vs scan_wpb=1 (one wave per block)
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t3.log
[ $rc -eq 0 ] || exit $rc
for v in default 1; do
  opt=""; [ "$v" != "default" ] && opt="--option scan_wpb=$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof3_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 $opt > gpurun_out/sprof3_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py gpurun_out/sprof3_$v | head -8
  grep -o '"search": {"metric[^}]*' gpurun_out/sprof3_$v.log | head -c 300; echo
done
