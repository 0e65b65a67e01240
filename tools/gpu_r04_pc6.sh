#!/bin/bash
# k_precomp_ws grid sizes (multiples of 1280 = 5 workgroups x 256 CUs) and non-temporal stores
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
for g in 12800 16384 20480 25600 32768 51200 65536; do pc grid$g $D HQ_PRECOMP_GRID=$g HQ_PRECOMP_NT=0 || exit 1; done
} | tee $O/pc6_ab.txt
