#!/bin/bash
# k_scanov: both blocks' contractions before the bounds (ov_mf) — parity under the option, then A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
D=$GRAFT_REPO_ROOT/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
HQ_LIB_VARIANT=$D HQ_OV_MF=1 HQ_OV_OCC=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_longlist.py tests/test_gpu_sortkey.py -q -x --timeout 300 --timeout-method thread -k "overall or brute or scanov or sort_key" > $O/ov3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/ov3_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, options...
  local tag=$1; shift
  local opts=""
  for o in "$@"; do opts="$opts --option $o"; done
  timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 $opts > $O/ov3_$tag.json 2> $O/ov3_$tag.err
  local rc=$?
  python3 -c "
import json,sys; d=json.loads(open('$O/ov3_$tag.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('%-10s search %.3fM  ov %.3fM  l0 %.3fM' % ('$tag', s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6))" || echo "$tag rc=$rc"
  return $rc
}
for rep in 1 2; do
  run new && run mf4 ov_mf=1 && run mf3 ov_mf=1 ov_occ=3 && run occ3 ov_occ=3 || exit 1
done
