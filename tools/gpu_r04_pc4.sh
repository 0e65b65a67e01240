#!/bin/bash
# k_precomp_ws: LDS footprint vs workgroups per CU (row pad 0 saves 1 KiB), grid A/B
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
for g in 1024 1280 2048 4096 8192; do pc pad0_grid$g $D HQ_PRECOMP_PAD=0 HQ_PRECOMP_GRID=$g || exit 1; done &&
pc pad4_grid1024 $D HQ_PRECOMP_GRID=1024
} | tee $O/pc4_ab.txt
