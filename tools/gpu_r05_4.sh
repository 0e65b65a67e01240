#!/bin/bash
# round 5, call 4: search legs only (cfg3 + modes + fresh / clustered) with the new re-rank and retry
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 500 python bench.py --no-stream --no-precomputed --no-ingest --no-frames --no-api --corpus-total 0 \
  --no-cpu > $O/r05_6_bench.json 2> $O/r05_6_bench.err; rc=$?; echo "bench rc=$rc"; exit $rc
