#!/bin/bash
# A/B the S7 MFMA cosine: each argument is a bench --option list ("-" = defaults), e.g. cos_kernel=3
for v in "$@"; do
  opts=""
  if [ "$v" != "-" ]; then for o in ${v//,/ }; do opts="$opts --option $o"; done; fi
  r=$(timeout -k 10 120 python bench.py --no-search --no-stream --no-precomputed --no-ingest --no-cpu --steps 2 $opts | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['frames']; print(round(d['value']/1e9,2), round(d['roofline']['achieved'],1), round(d['roofline']['frac'],3), round(d['ms_per_step'],3))") || exit 1
  echo "$v: $r"
done
