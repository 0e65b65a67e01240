#!/bin/bash
# k_precomp_ws phase costs (DIAG library: 1 skip small squares, 2 skip leaves, 8 skip stores) and grid A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
pc() {  # tag, env...
  local tag=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 2>$O/pc_$tag.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))") || { echo "$tag failed"; tail -3 $O/pc_$tag.err; return 1; }
  echo "$tag: $r"
}
D=HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
{
pc default HQ_NONE=1 &&
for v in 1 2 8 3 9 10 11; do pc diag$v $D HQ_PRECOMP_DIAG=$v || exit 1; done &&
for g in 1280 2560 3840 5120 16384; do pc grid$g $D HQ_PRECOMP_GRID=$g || exit 1; done &&
pc nt0 $D HQ_PRECOMP_NT=0
} | tee $O/pc3_ab.txt
