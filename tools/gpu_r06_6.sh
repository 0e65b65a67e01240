#!/bin/bash
# checkpoint: whole GPU suite, smoke, default bench, bench kernel statistics; the sample pass's one-round-trip
# epilogue (kernel statistics of the M = 20 search), the cold clustered batch with the redo warm-up
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
V=${1:-v2}
mkdir -p $O
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof6_m20 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py m20 > $O/prof6_m20.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "prof rc=$rc"; tail -5 $O/prof6_m20.log; exit $rc; }
python3 tools/prof_summary.py $O/prof6_m20 | grep -E "sample|scan0g|rank_small|pool_select|prepare" 
timeout -k 10 300 python tools/cold_batch_prof.py > $O/r06_6_cold.log 2>&1; echo "cold rc=$?"; grep -E "batch:" $O/r06_6_cold.log
bash tools/gpu_r06_full.sh $V
