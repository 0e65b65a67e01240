#!/bin/bash
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/pc_stride.py 2>$O/pcs.err || { echo "rc=$?"; tail -5 $O/pcs.err; exit 1; }
