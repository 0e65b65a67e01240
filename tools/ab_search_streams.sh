#!/bin/bash
# A/B the search leg over HQ_SEARCH_STREAMS (streams the in-flight batches alternate over), 2 rounds
for rep in 1 2; do
for n in "$@"; do
  r=$(HQ_SEARCH_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu --no-ingest --no-frames --no-precomputed --no-stream --steps 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['search']; print(round(d['value']), round(d['ms_per_step'], 4), d['self_match_rate'])") || exit 1
  echo "streams=$n: $r"
done
done
