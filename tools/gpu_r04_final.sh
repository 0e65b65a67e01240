#!/bin/bash
# final binary sanity: smoke + search / long-list GPU tests
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/fin_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/fin_smoke.log; exit 1; }
tail -1 $O/fin_smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_longlist.py tests/test_gpu_search.py tests/test_gpu_precomputed.py -q -x --timeout 300 --timeout-method thread > $O/fin_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/fin_tests.log; exit $rc
