#!/bin/bash
# default bench (search legs at 50 batches)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
T0=$(date +%s); timeout -k 10 500 python bench.py > $O/r05_27_bench.json 2> $O/r05_27_bench.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - T0 ))s"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads(open('$O/r05_27_bench.json').read().strip().splitlines()[-1]); s=d['search']
print(round(d['value']/1e6,1), 'search', round(s['value']/1e6,3), 'ms', s['ms_per_step']); [print(k, round(v['value']/1e6,3)) for k,v in s.get('modes',{}).items() if 'value' in v]"
