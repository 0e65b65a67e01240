#!/bin/bash
# redo count read "async" (copy queued at submit on a side stream behind the re-rank's event): tests, A/B vs copy
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hard_queries.py::test_redo_count_read_modes > $O/r06_19_tests.log 2>&1 || { tail -30 $O/r06_19_tests.log; exit 1; }
tail -3 $O/r06_19_tests.log
E="--py-set hq_mi355x.core.search_engine:IndexCorpus._count_read=async"
bash tools/ab_bench_search.sh r06_19_ab "copy|" "async|$E" || exit 1
