#!/bin/bash
# A/B the pre-computed index leg over env assignment lists ("-" = defaults), 2 rounds
for rep in 1 2; do
for v in "$@"; do
  [ "$v" = "-" ] && v="HQ_NONE=1"
  r=$(env $v timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['ms_per_step'],3))") || exit 1
  echo "$v: $r"
done
done
