#!/bin/bash
# k_sample_kth register pool per size (parity + time); k_refine_lds phase split (DIAG expt 1: no staging, 2: no scoring)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_f32.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_t19a.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -2 gpurun_out/r03_t19a.log; [ $rc -eq 0 ] || exit $rc
DIAG=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for e in 0 1 2; do
  HQ_LIB_VARIANT=$DIAG HQ_REFINE_EXPT=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_19_$e -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 > gpurun_out/prof_r03_19_$e.log 2>&1 || exit 1
  echo "== refine expt $e"; python3 tools/prof_summary.py gpurun_out/prof_r03_19_$e | grep -E "k_refine_lds|k_sample_kth|k_scan0g|k_sample_topg"
done
