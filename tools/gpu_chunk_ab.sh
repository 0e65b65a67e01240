#!/bin/bash
# cfg5 chunk encoder: parity tests, then the stream leg of the bench (kernel time under rocprof)
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest $(grep -ln "chunk_encode" tests/test_gpu_*.py) -q -x --timeout 500 --timeout-method thread > gpurun_out/chunk_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/chunk_t.log
[ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  opts=""; for o in ${spec//,/ }; do [ "$o" != "default" ] && opts="$opts --option $o"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cab -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-search --no-precomputed --no-ingest --no-frames $opts > gpurun_out/cab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -3 gpurun_out/cab.log; exit $rc; }
  echo "[$spec] $(python3 tools/prof_summary.py gpurun_out/cab | grep -E 'k_chunk_np' | tr -s ' ' | cut -c1-100) $(grep -o '"stream": {"metric[^}]*' gpurun_out/cab.log | grep -o '"value": [0-9.]*')"
done
