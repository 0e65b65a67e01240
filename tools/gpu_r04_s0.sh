#!/bin/bash
# level-0 scan with LDS-buffered pool appends: search parity tests, then A/B of the search leg vs the
# previous head's library (.baseline_pc/)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_longlist.py tests/test_gpu_sortkey.py tests/test_gpu_search_f32.py tests/test_gpu_api_golden.py tests/test_gpu_diag_bounds.py -q -x --timeout 300 --timeout-method thread > $O/s0_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/s0_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, env/options...
  local tag=$1; shift
  local env=""; local opts=""
  for o in "$@"; do case $o in HQ_*) env="$env $o";; *) opts="$opts --option $o";; esac; done
  env $env timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 $opts > $O/s0_$tag.json 2> $O/s0_$tag.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads(open('$O/s0_$tag.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('%-10s search %.3fM  ov %.3fM  l0 %.3fM  m100 %.3fM  m1000 %.3fM' % ('$tag', s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6, m['m100']['value']/1e6, m['m1000']['value']/1e6))" || echo "$tag rc=$rc"
  return $rc
}
run new && run old HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/.baseline_pc/libhq_mi355x.so && run new2 && run old2 HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/.baseline_pc/libhq_mi355x.so
