#!/bin/bash
# bench search legs: SEARCH_DEPTH 3 (default now) vs 2, m100 / m1000 pipelined; 200 search steps
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
B="--corpus-total 0 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --no-hard --no-api --steps 3 --warmup 1"
for rep in 1 2; do
for d in 3 2; do
  HQ_SEARCH_DEPTH=$d timeout -k 10 300 python bench.py $B > $O/r06_17_d${d}_$rep.json 2> $O/r06_17_d${d}_$rep.err || { tail -5 $O/r06_17_d${d}_$rep.err; exit 1; }
  F=$O/r06_17_d${d}_$rep.json D=$d python3 -c "
import json, os; d=json.loads(open(os.environ['F']).read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('depth', os.environ['D'], 'm20', round(s['value']/1e6,3), 'm100', round(m['m100']['value']/1e6,3), '(sync', round(m['m100']['sync']['value']/1e6,3), ') m1000', round(m['m1000']['value']/1e6,3), '(sync', round(m['m1000']['sync']['value']/1e6,3), ') overall', round(m['overall']['value']/1e6,3))"
done; done
