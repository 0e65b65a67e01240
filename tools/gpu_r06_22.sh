#!/bin/bash
# kernel times of the M = 100 / 1000 searches with and without the window ranking (tools/scan_debug.py)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for w in 1 0; do for m in m100 m1000; do
  cd /tmp && HQ_DBG_OPTS=rank_win=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r06_22_w${w}_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py $m > $O/r06_22_w${w}_$m.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT; echo "rank_win=$w $m"; python3 tools/prof_summary.py $O/r06_22_w${w}_$m | grep -E "k_rank|k_pool|k_scan0g|k_sample" | head -8
done; done
