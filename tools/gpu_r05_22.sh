#!/bin/bash
# M = 20 progressive: fused short-list re-rank (default) against k_refine_lds (refine_small = 0)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for v in 1 0; do
  cd /tmp && HQ_DBG_OPTS=refine_small=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof22_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py m20 > $O/prof22_$v.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; echo "refine_small=$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py $O/prof22_$v > $O/prof22_$v.txt; grep -E "scan0g|rank_|refine|pool_s|final|sample|prepare" $O/prof22_$v.txt
done
