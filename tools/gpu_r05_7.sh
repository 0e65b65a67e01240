#!/bin/bash
# round 5, call 7: compact pre-computed averages (6 workgroups per CU): parity + A/B of the precomputed leg
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_precomputed.py -x -q --timeout 300 --timeout-method thread > $O/r05_7_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r05_7_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for opt in 1 0; do
timeout -k 10 200 python bench.py --no-search --no-stream --no-ingest --no-frames --no-api --no-cpu --steps 4 --option precomp_compact=$opt > $O/r05_7_pc$opt.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads(open('$O/r05_7_pc$opt.json').read().strip().splitlines()[-1]); p=r['precomputed']; print('compact=$opt', round(p['value']/1e6,1), 'M emb/s frac', round(p['roofline']['frac'],4), 'kernel ms', round(p['roofline']['kernel_ms'],3))"
done; done
