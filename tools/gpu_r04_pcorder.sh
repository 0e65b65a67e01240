#!/bin/bash
# pre-computed index kernel time in the bench: alone after the headline vs after the search legs
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
pc() {  # tag, bench args...
  local tag=$1; shift
  r=$(timeout -k 10 300 python bench.py --no-stream --no-cpu --no-ingest --no-frames "$@" 2>$O/pco_$tag.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3))") || { echo "$tag failed"; tail -3 $O/pco_$tag.err; return 1; }
  echo "$tag: $r"
}
for rep in 1 2; do
  pc alone --no-search --steps 20 || exit 1
  pc after_search --steps 20 || exit 1
  pc after_search_nostrong --steps 20 --corpus-total 0 || exit 1
done
