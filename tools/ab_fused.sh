#!/bin/bash
# A/B the fused-kernel variants (HQ_FUSED_V bitmask: 1 nt loads, 2 fast quantize, 4 triple buffer)
for v in "$@"; do
  r=$(HQ_FUSED_V=$v timeout -k 10 120 python bench.py --no-search --no-stream --no-precomputed --no-ingest --no-frames --no-cpu --steps 30 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['roofline']['frac'],3))") || exit 1
  echo "V=$v: $r"
done
