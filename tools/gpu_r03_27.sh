#!/bin/bash
# search A/B: statistical starting threshold K' (option sample_kth) 12 (default) vs 10 vs 11
export TMPDIR=/tmp
for o in - sample_kth=10 sample_kth=11 - sample_kth=10 sample_kth=11 - sample_kth=10; do
  opts=""; [ "$o" != "-" ] && opts="--option $o"
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 60 $opts > gpurun_out/r03_s27.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_s27.json'))['search']; print('$o', round(d['value']/1e6,3), 'M QPS', round(d['ms_per_step'],4), 'ms/step')"
done
