#!/bin/bash
# bench with the pre-computed leg moved next to the headline: every leg's number, twice
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu --no-ingest > $O/pco2_$rep.json 2>$O/pco2_$rep.err || { echo "bench rc=$?"; tail -5 $O/pco2_$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/pco2_$rep.json')); s=d['search']
print('head', round(d['value']/1e6,1), 'pre', round(d['precomputed']['value']/1e6,1), round(d['precomputed']['roofline']['kernel_ms'],3),
      'search', round(s['value']/1e6,3), 'strong', round(s['strong']['value']/1e6,3), {k: round(v['value']/1e6,3) for k, v in s['modes'].items()},
      'frames', round(d['frames']['value']/1e9,2), 'stream', round(d['stream']['value'],0))"
done
