#!/bin/bash
# search: corpus flag list precomputed, query overall layout on demand, batches in flight 2 vs 3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py tests/test_gpu_diag_bounds.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t15a.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -3 gpurun_out/r03_t15a.log; [ $rc -eq 0 ] || exit $rc
for d in 2 3 2 3; do
  HQ_SEARCH_DEPTH=$d timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 40 > gpurun_out/r03_s15_$d.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_s15_$d.json'))['search']; print('depth $d', round(d['value']/1e6,3), 'M QPS', round(d['ms_per_step'],4), 'ms/step;', {k: round(v['value']/1e6,3) for k, v in d['modes'].items()})"
done
