#!/bin/bash
# the redo count published by the re-rank kernel (count_read "kernel"): parity tests, then A/B against the
# pinned copy; k_rank_small at 3 waves per SIMD (rank_occ 3, no spill); sample_waves; k_scanov ov_occ 3 + ov_pf
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hard_queries.py::test_redo_count_read_modes tests/test_gpu_threads.py > $O/r06_14_tests.log 2>&1 || { tail -30 $O/r06_14_tests.log; exit 1; }
tail -3 $O/r06_14_tests.log
E="--py-set hq_mi355x.core.search_engine:IndexCorpus._count_read=kernel"
bash tools/ab_bench_search.sh r06_14_ab "copy|" "kernel|$E" "kernel rank_occ=3|$E --option rank_occ=3" "sample_waves=4096|--option sample_waves=4096" "ov_occ=3 ov_pf=2|--option ov_occ=3 --option ov_pf=2" "ov_occ=3 ov_pf=3|--option ov_occ=3 --option ov_pf=3" || exit 1
