#!/bin/bash
# k_precomp_ws: phase costs (DIAG: 1 small squares, 2 leaves, 8 stores) and PMC passes
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
for v in 1 2 8 3 9 10 11; do pc diag$v $D HQ_PRECOMP_DIAG=$v || exit 1; done
} | tee $O/pc5_ab.txt || exit 1
bash tools/pmc_lds.sh precomp5 --no-search --no-stream --no-ingest --no-frames
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/pmc_precomp5/summary.txt')) if False else None
PY
cat gpurun_out/pmc_precomp5/summary.txt | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
for k,v in d.items():
    if 'precomp' in k: print(k, json.dumps(v)[:1500])"
