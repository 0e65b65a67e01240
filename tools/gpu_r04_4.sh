#!/bin/bash
# long-list re-rank rewrite + sample passes back on the split form: targeted tests, then the scan A/B,
# then PMC of the level-0 scan (hi.hi default and the three-MFMA form)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_sortkey.py tests/test_gpu_search_f32.py -q -x --timeout 300 --timeout-method thread > $O/r04_t4.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/r04_t4.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04_ab1.sh || exit 1
bash tools/pmc_kernel.sh k_scan0g $O/pmc_scan0g_hi level0 || exit 1
HQ_DBG_OPTS=scan_split3=1 bash tools/pmc_kernel.sh k_scan0g $O/pmc_scan0g_s3 level0 || exit 1
bash tools/pmc_kernel.sh k_scanov $O/pmc_scanov_hi overall || exit 1
