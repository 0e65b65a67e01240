#!/bin/bash
# diagnostics build: k_scan0g time at list lengths 28 / 108 / 1008 with the pool append as is (0), without the
# atomic's return value (10) and without any append (11)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export HQ_LIB_VARIANT=$GRAFT_REPO_ROOT/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for k in 28 108 1008; do for e in 0 10 11; do
  cd /tmp && HQ_DBG_OPTS=scan_expt=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p16_${k}_$e -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scan_debug.py scan$k > $O/p16_${k}_$e.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { echo "k=$k e=$e rc=$rc"; tail -5 $O/p16_${k}_$e.log; exit $rc; }
  echo "k=$k expt=$e $(python3 tools/prof_summary.py $O/p16_${k}_$e | grep -E 'k_scan0g')"
done; done
