# round-3 GPU check: search tests first (new k_scan0g), then the whole GPU suite, then the bench
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_search.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -3 gpurun_out/r03_search.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03_t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r03_b1.json 2> gpurun_out/r03_b1.err
echo "bench rc=$?"
