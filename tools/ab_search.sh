#!/bin/bash
# A/B search knobs: each argument is an env assignment list (e.g. "HQ_SAMPLE_STRIDE=32"); "-" = defaults
for v in "$@"; do
  [ "$v" = "-" ] && v="HQ_NONE=1"
  r=$(env $v timeout -k 10 120 python bench.py --no-stream --no-cpu --steps 2 --warmup 1 --search-steps 10 | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['search']; print(round(d['value']), round(d['ms_per_step'],3))") || exit 1
  echo "$v: $r"
done
