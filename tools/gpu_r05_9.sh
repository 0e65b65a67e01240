#!/bin/bash
# round 5, call 9: A/B of the sample stride on the cfg3 search leg (and its modes)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for i in 1 2; do
for st in 16 32 8; do
timeout -k 10 300 python bench.py --no-precomputed --no-stream --no-ingest --no-frames --no-api --no-hard --no-cpu --corpus-total 0 --steps 2 --option sample_stride=$st > $O/r05_9_s$st.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads(open('$O/r05_9_s$st.json').read().strip().splitlines()[-1]); s=r['search']; m=s['modes']; print('stride $st', round(s['value']/1e6,3), 'overall', round(m['overall']['value']/1e6,3), 'm100', round(m['m100']['value']/1e6,3), 'm1000', round(m['m1000']['value']/1e6,3), 'level0', round(m['level0']['value']/1e6,3))"
done; done
