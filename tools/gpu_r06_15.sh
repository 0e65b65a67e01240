#!/bin/bash
# the redo flags stored to pinned host memory by the re-rank kernel, per query (count_read "kernel"): parity
# tests, then A/B against the pinned copy of the count
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O


E="--py-set hq_mi355x.core.search_engine:IndexCorpus._count_read=kernel"
bash tools/ab_bench_search.sh r06_16_ab "copy|" "kernel flags|$E" "kernel flags unchecked|$E --py-set hq_mi355x.core.search_engine:IndexCorpus._check_flags=0" || exit 1
