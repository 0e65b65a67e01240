# GPU suite + search-leg kernel profiles, default scan vs the list-based k_scan0f (scan_variant=1)
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/r03_t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in default 1; do
  opt=""; [ "$v" != "default" ] && opt="--option scan_variant=$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 $opt > gpurun_out/sprof_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
