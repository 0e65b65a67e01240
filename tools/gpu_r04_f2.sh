#!/bin/bash
# long-list re-rank with one-pass correlation + mse sums: search parity tests, search-leg bench, kernel trace
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_search_f32.py tests/test_gpu_sortkey.py tests/test_gpu_api_golden.py -q -x --timeout 300 --timeout-method thread > $O/f2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/f2_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-precomputed --no-frames --no-ingest --no-stream --corpus-total 0 --steps 3 --search-steps 20 > $O/f2_b$rep.json 2> $O/f2_b$rep.err || { echo "bench rc=$?"; tail -3 $O/f2_b$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/f2_b$rep.json').read().strip().splitlines()[-1]); s=d['search']; m=s['modes']
print('search %.3fM ov %.3fM l0 %.3fM m100 %.3fM m1000 %.3fM' % (s['value']/1e6, m['overall']['value']/1e6, m['level0']['value']/1e6, m['m100']['value']/1e6, m['m1000']['value']/1e6))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py m1000 > $O/prof_f2.log 2>&1 || { echo "prof rc=$?"; tail -3 $O/prof_f2.log; exit 1; }
f=$(ls $O/prof_f2/*/run_kernel_stats.csv $O/prof_f2/run_kernel_stats.csv 2>/dev/null | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('refine', 'pool_sort', 'scan0g', 'sample')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')"
