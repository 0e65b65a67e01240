#!/bin/bash
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/clustered_prof.py > $O/r05_5.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r05_5.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r05_5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/clustered_prof.py > $O/r05_5_prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; python3 tools/prof_summary.py $O/prof_r05_5; exit $rc
