#!/bin/bash
# k_scanov drain gate: overall / brute-force parity tests, then A/B of the search leg vs the previous library
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_longlist.py tests/test_gpu_sortkey.py -q -x --timeout 300 --timeout-method thread -k "overall or brute or scanov or sort_key" > $O/ov1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ov1_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, env/options...
  local tag=$1; shift
  local env=""; local opts=""
  for o in "$@"; do case $o in HQ_*) env="$env $o";; *) opts="$opts --option $o";; esac; done
  env $env timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 $opts > $O/ov1_$tag.json 2> $O/ov1_$tag.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads(open('$O/ov1_$tag.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('%-10s search %.3fM  ov %.3fM  l0 %.3fM  m100 %.3fM  m1000 %.3fM' % ('$tag', s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6, m['m100']['value']/1e6, m['m1000']['value']/1e6))" || echo "$tag rc=$rc"
  return $rc
}
run new && run w8k ov_waves=8192 && run w16k ov_waves=16384 && run w32k ov_waves=32768 && run new2
