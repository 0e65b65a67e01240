#!/bin/bash
# round 5, call 3: pair-scoring + sort re-rank (k_rank_pairs / k_rank_sort): long-list parity, timing vs the
# per-thread kernels, hard query tests
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_longlist.py -x -q --timeout 300 --timeout-method thread > $O/r05_3_longlist.log 2>&1
rc=$?; echo "longlist rc=$rc"; tail -3 $O/r05_3_longlist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/refine_timing.py > $O/r05_3_refine.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r05_3_refine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_hard_queries.py -x -v -s --timeout 600 --timeout-method thread > $O/r05_3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "M=|passed|failed|Error" $O/r05_3_tests.log | head -20; exit $rc
