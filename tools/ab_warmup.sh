#!/bin/bash
# headline rate vs warmup / step count (clock ramp check)
for a in "--warmup 3 --steps 20" "--warmup 500 --steps 20" "--warmup 1500 --steps 20" "--warmup 3 --steps 1000"; do
  r=$(timeout -k 10 120 python bench.py --no-search --no-stream --no-precomputed --no-frames --no-ingest --no-cpu $a | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['roofline']['achieved'],0), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))") || exit 1
  echo "$a: $r"
done
