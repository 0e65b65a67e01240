#!/bin/bash
# k_scan0g with 128-query waves (option scan_nb 8): parity, then search A/B interleaved
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_diag_bounds.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t22a.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -2 gpurun_out/r03_t22a.log; [ $rc -eq 0 ] || exit $rc
for o in - scan_nb=8 - scan_nb=8 - scan_nb=8; do
  opts=""; [ "$o" != "-" ] && opts="--option $o"
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 40 $opts > gpurun_out/r03_s22.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_s22.json'))['search']; print('$o', round(d['value']/1e6,3), 'M QPS', round(d['ms_per_step'],4), 'ms/step;', {k: round(v['value']/1e6,3) for k, v in d['modes'].items()})"
done
