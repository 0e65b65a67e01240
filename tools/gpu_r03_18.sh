#!/bin/bash
# search A/B: sample pass waves (option sample_waves), 3 runs each interleaved
export TMPDIR=/tmp
for o in - sample_waves=4096 sample_waves=1024 - sample_waves=4096 sample_waves=1024; do
  opts=""; [ "$o" != "-" ] && opts="--option $o"
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 40 $opts > gpurun_out/r03_s18.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_s18.json'))['search']; print('$o', round(d['value']/1e6,3), 'M QPS', round(d['ms_per_step'],4), 'ms/step')"
done
