#!/bin/bash
# PMC passes of the M = 20 batch's kernels (k_rank_small, k_scan0g, k_pool_select, k_sample_kth)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for k in k_rank_small k_scan0g k_sample_kth k_pool_select; do
  timeout -k 10 300 bash tools/pmc_kernel.sh $k $O/r06_8_pmc_$k m20 > $O/r06_8_pmc_$k.txt 2>&1; rc=$?; echo "pmc $k rc=$rc"; tail -3 $O/r06_8_pmc_$k.txt | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done
