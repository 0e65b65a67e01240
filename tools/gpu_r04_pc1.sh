#!/bin/bash
# k_precomp (cfg: 1M x 1536-d f32 -> 64x64, zero-padding skip): phase costs (DIAG library), grid / pad A/B,
# LDS PMC passes
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
pc() {  # tag, env..., -- bench options
  local tag=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 2>$O/pc_$tag.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['ms_per_step'],3))") || { echo "$tag failed"; tail -3 $O/pc_$tag.err; return 1; }
  echo "$tag: $r"
}
D=HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
{
pc default HQ_NONE=1 &&
for v in 0 1 2 4 8 3 5 6 9 7 15; do pc diag$v $D HQ_PRECOMP_DIAG=$v || exit 1; done &&
for g in 2048 4096 16384 32768; do pc grid$g $D HQ_PRECOMP_GRID=$g || exit 1; done &&
for p in 0 8 12; do pc pad$p $D HQ_PRECOMP_PAD=$p || exit 1; done
} | tee $O/pc1_ab.txt || exit 1
bash tools/pmc_lds.sh precomp --no-search --no-stream --no-ingest --no-frames
cat gpurun_out/pmc_precomp/summary.txt | head -40
