#!/bin/bash
# refine at 4 waves/SIMD (k_refine_lds_sm) + kth register pools: search parity, then search bench x3 and kernel times
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py tests/test_gpu_ingest.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t20a.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -2 gpurun_out/r03_t20a.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 40 > gpurun_out/r03_s20.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_s20.json'))['search']; print('run $i', round(d['value']/1e6,3), 'M QPS', round(d['ms_per_step'],4), 'ms/step;', {k: round(v['value']/1e6,3) for k, v in d['modes'].items()})"
done
bash tools/search_only_prof.sh r03u > gpurun_out/r03_sprof20.txt 2>&1; rc=$?; head -16 gpurun_out/r03_sprof20.txt
python3 tools/trace_gaps.py gpurun_out/sprof_r03u k_sample_topg 10 k_sampleov
exit $rc
