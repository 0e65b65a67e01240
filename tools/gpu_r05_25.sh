#!/bin/bash
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 200 python tools/host_overhead.py 20 > $O/r05_25.log 2>&1; rc=$?; grep -v amdgpu.ids $O/r05_25.log | head -60; exit $rc
