set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_search_f32.py tests/test_gpu_search.py -m gpu > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -30 gpurun_out/f32_tests.log
exit $rc
