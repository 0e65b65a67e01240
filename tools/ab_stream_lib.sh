#!/bin/bash
# A/B the cfg5 stream leg between the in-tree library ("-") and variant builds (HQ_LIB_VARIANT), 3 rounds
for rep in 1 2 3; do
for v in "$@"; do
  if [ "$v" = "-" ]; then e="HQ_NONE=1"; else e="HQ_LIB_VARIANT=$v"; fi
  r=$(env $e timeout -k 10 120 python bench.py --no-search --no-cpu --no-precomputed --no-frames --no-ingest --steps 5 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['stream']; print(round(d['value'],1), round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],3))") || exit 1
  echo "$v: $r"
done
done
