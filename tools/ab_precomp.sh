#!/bin/bash
# A/B the pre-computed index kernel: each argument is an env assignment list ("-" = defaults)
for v in "$@"; do
  [ "$v" = "-" ] && v="HQ_NONE=1"
  r=$(env $v timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['roofline']['frac'],3))") || exit 1
  echo "$v: $r"
done
