#!/bin/bash
# A/B of the hi.hi scans (search leg only, one box): default, three-MFMA forms, register targets
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
run() {  # tag, options...
  local tag=$1; shift
  local opts=""
  for o in "$@"; do opts="$opts --option $o"; done
  timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 $opts > $O/ab1_$tag.json 2> $O/ab1_$tag.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads(open('$O/ab1_$tag.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('%-14s search %.3fM  ov %.3fM  l0 %.3fM  m100 %.3fM  m1000 %.3fM' % ('$tag', s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6, m['m100']['value']/1e6, m['m1000']['value']/1e6))" || echo "$tag rc=$rc"
  return $rc
}
run default && run split3 scan_split3=1 scanov_split3=1 ov_occ=2 && run occ4 scan_occ=4 ov_occ=3 && run occ6 scan_occ=6 && run ovocc2 ov_occ=2 && run default2
