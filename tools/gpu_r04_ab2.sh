#!/bin/bash
# A/B of the level-0 scan's prefetch distance / occupancy / queries per wave (search leg only, one box)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
run() {  # tag, options...
  local tag=$1; shift
  local opts=""
  for o in "$@"; do opts="$opts --option $o"; done
  timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 $opts > $O/ab2_$tag.json 2> $O/ab2_$tag.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads(open('$O/ab2_$tag.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('%-14s search %.3fM  ov %.3fM  l0 %.3fM  m100 %.3fM  m1000 %.3fM' % ('$tag', s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6, m['m100']['value']/1e6, m['m1000']['value']/1e6))" || echo "$tag rc=$rc"
  return $rc
}
run default && run pf3 scan_pf=3 && run pf4 scan_pf=4 && run pf6 scan_pf=6 && run occ5 scan_occ=5 && run nb8 scan_nb=8 && run default2
