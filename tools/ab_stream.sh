#!/bin/bash
# A/B the cfg5 chunk-encoder launch forms: each argument is an env assignment list, e.g. "HQ_CHUNK_WPB=4"
for v in "$@"; do
  [ "$v" = "-" ] && v="HQ_NONE=1"
  r=$(env $v timeout -k 10 120 python bench.py --no-search --no-cpu --no-precomputed --no-frames --no-ingest --steps 2 --warmup 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['stream']; print(round(d['value'],1), round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],3))") || exit 1
  echo "$v: $r"
done
