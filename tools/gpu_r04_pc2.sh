#!/bin/bash
# k_precomp: parity tests + A/B of the current library against the previous one (saved under .baseline_pc/)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_precomputed.py -q -x --timeout 200 --timeout-method thread > $O/pc2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pc2_tests.log; [ $rc -eq 0 ] || exit $rc
pc() {  # tag, env...
  local tag=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 2>$O/pc_$tag.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))") || { echo "$tag failed"; tail -3 $O/pc_$tag.err; return 1; }
  echo "$tag: $r"
}
for rep in 1 2; do
  pc new HQ_NONE=1 || exit 1
  D=HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
  pc nows $D HQ_PRECOMP_WS=0 || exit 1
  pc lw3 $D HQ_PRECOMP_WS=3 || exit 1
  [ -f .baseline_pc/libhq_mi355x.so ] && { pc old HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/.baseline_pc/libhq_mi355x.so || exit 1; }
done
