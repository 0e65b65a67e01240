#!/bin/bash
# drain gate + PF / OCC options + fused query prep + ping-pong redo counter: targeted tests, A/B, full bench + trace
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py tests/test_gpu_search_f32.py tests/test_gpu_distributed.py -q -x --timeout 300 --timeout-method thread > $O/r04_t5.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/r04_t5.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04_ab2.sh || exit 1
timeout -k 10 400 python bench.py --no-cpu > $O/r04_b5.json 2> $O/r04_b5.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_r04b5 -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > $O/prof_r04b5.log 2>&1
rc=$?; echo "prof rc=$rc"; python3 tools/prof_summary.py $O/prof_r04b5 | head -24; exit $rc
