#!/bin/bash
# fused final ranking for short lists: tests, statistics, bench
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_hard_queries.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py tests/test_gpu_sortkey.py tests/test_gpu_api_golden.py -x -q --timeout 300 --timeout-method thread > $O/r05_26_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r05_26_tests.log; [ $rc -eq 0 ] || exit $rc
for m in m20 m100 m1000; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof26_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/prof26_$m.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; echo "prof $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py $O/prof26_$m > $O/prof26_$m.txt; grep -E "scan0g|rank_|refine|pool_s|final|sample_topg" $O/prof26_$m.txt
done
timeout -k 10 300 python bench.py --no-cpu --no-hard --no-api > $O/r05_26_bench.json 2> $O/r05_26_bench.err; rc=$?; echo "bench rc=$rc"
python3 -c "
import json; d=json.loads(open('$O/r05_26_bench.json').read().strip().splitlines()[-1]); s=d['search']
print('search', round(s['value']/1e6,3), 'M', s['ms_per_step']); [print(k, round(v['value']/1e6,3)) for k,v in s.get('modes',{}).items() if 'value' in v]"
timeout -k 10 200 python tools/host_overhead.py 20 > $O/r05_26_host.log 2>&1; head -1 $O/r05_26_host.log
