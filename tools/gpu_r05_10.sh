#!/bin/bash
# round 5, call 10: cooperative query preparation parity + search tests, then the sample-stride A/B
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_search_f32.py -x -q --timeout 300 --timeout-method thread > $O/r05_10_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r05_10_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for st in 16 32; do
timeout -k 10 300 python bench.py --no-precomputed --no-stream --no-ingest --no-frames --no-api --no-hard --no-cpu --corpus-total 0 --steps 2 --option sample_stride=$st > $O/r05_10_s$st.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads(open('$O/r05_10_s$st.json').read().strip().splitlines()[-1]); s=r['search']; m=s['modes']; print('stride $st', round(s['value']/1e6,3), 'overall', round(m['overall']['value']/1e6,3), 'm100', round(m['m100']['value']/1e6,3), 'm1000', round(m['m1000']['value']/1e6,3), 'level0', round(m['level0']['value']/1e6,3))"
done; done
timeout -k 10 300 python bench.py --no-precomputed --no-stream --no-ingest --no-frames --no-api --no-hard --no-cpu --no-modes --corpus-total 0 --steps 2 --option prep_coop=0 > $O/r05_10_p0.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads(open('$O/r05_10_p0.json').read().strip().splitlines()[-1]); s=r['search']; print('prep_coop=0', round(s['value']/1e6,3))"
