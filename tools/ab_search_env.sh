#!/bin/bash
# A/B of search-only bench lines under different environment settings, one box.
# usage: tools/ab_search_env.sh "HQ_SAMPLE_STRIDE=16" "HQ_SAMPLE_STRIDE=32" ...
OUT=gpurun_out; mkdir -p $OUT
i=0
for rep in 1 2; do
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 > $OUT/ab_s_$i.json 2> $OUT/ab_s_$i.err || { echo "fail: $e"; tail -3 $OUT/ab_s_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab_s_$i.json'));s=d['search'];print('$e', round(s['value']), round(s['ms_per_step'],4))"
done
done
