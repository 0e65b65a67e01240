#!/bin/bash
# A/B: redo count read (pinned copy on the search stream vs event + side-stream read), sample stride; tests first
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_search.py tests/test_gpu_longlist.py tests/test_gpu_hard_queries.py -x -q --timeout 300 --timeout-method thread > $O/r06_2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r06_2_tests.log; [ $rc -eq 0 ] || exit $rc
B="--corpus-total 0 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --no-hard --no-api --steps 3 --warmup 1"
i=0
for rep in 1 2; do
for v in "IndexCorpus._count_read = 'copy'|" "IndexCorpus._count_read = 'side'|" "IndexCorpus._count_read = 'side'|--option sample_stride=32" "IndexCorpus._count_read = 'side'|--option sample_stride=8" "IndexCorpus._count_read = 'side'|--option rank_e=2" "IndexCorpus._count_read = 'side'|--option rank_e=4"; do
  i=$((i+1)); py="${v%%|*}"; opt="${v#*|}"
  timeout -k 10 300 python tools/ab_py.py "$py" $B $opt > $O/r06_2_ab_$i.json 2> $O/r06_2_ab_$i.err || { echo "fail: $v"; tail -3 $O/r06_2_ab_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/r06_2_ab_$i.json').read().strip().splitlines()[-1]); s=d['search']; m=s.get('modes',{})
print('$v', 'm20', round(s['value']/1e6,3), 'm100', round(m['m100']['value']/1e6,3), 'm1000', round(m['m1000']['value']/1e6,3), 'ov', round(m['overall']['value']/1e6,3), 'strong', round(s.get('strong',{}).get('value',0)/1e6,3))"
done; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r06_2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py m20 > $O/prof_r06_2.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_gaps.py $O/prof_r06_2 k_seg_prepare_pack0 10 > $O/r06_2_step.txt; cat $O/r06_2_step.txt
timeout -k 10 300 python tools/clustered_prof.py > $O/r06_2_clustered.log 2>&1; echo "clustered rc=$?"; cat $O/r06_2_clustered.log | tail -12
