#!/bin/bash
# A/B of the bench's search legs (cfg3 corpus, modes; no cfg4 strong leg) over kernel options, two reps, one
# box.  usage: tools/ab_bench_search.sh <tag> "<label>|<bench args>[|<library variant .so>]" ...
# (results: gpurun_out/<tag>_*.json; a variant library is loaded through HQ_LIB_VARIANT)
O=$GRAFT_REPO_ROOT/gpurun_out
tag=$1; shift
B="--corpus-total 0 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --no-hard --no-api --steps 3 --warmup 1"
i=0
for rep in 1 2; do
for v in "$@"; do
  i=$((i+1)); label="${v%%|*}"; rest="${v#*|}"; args="${rest%%|*}"; lib=""
  [ "$rest" != "$args" ] && lib="${rest#*|}"
  HQ_LIB_VARIANT=$lib timeout -k 10 300 python bench.py $B $args > $O/${tag}_$i.json 2> $O/${tag}_$i.err || { echo "fail: $v"; tail -3 $O/${tag}_$i.err; exit 1; }
  LABEL="$label" F="$O/${tag}_$i.json" python3 -c "
import json, os; d=json.loads(open(os.environ['F']).read().strip().splitlines()[-1]); s=d['search']; m=s.get('modes',{})
print(os.environ['LABEL'].ljust(28), 'm20', round(s['value']/1e6,3), 'm100', round(m['m100']['value']/1e6,3), 'm1000', round(m['m1000']['value']/1e6,3), 'overall', round(m['overall']['value']/1e6,3), 'level0', round(m['level0']['value']/1e6,3))"
done; done
