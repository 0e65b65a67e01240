#!/bin/bash
# float32 cosine scores: tests, frames leg, PMC traffic of the float32 kernel
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -q -x --timeout 200 --timeout-method thread -k cosine > $O/cos_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/cos_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-search --no-precomputed --no-stream --no-ingest --no-cpu --steps 3 > $O/cos_bench.json 2>$O/cos_bench.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/cos_bench.json').read().strip().splitlines()[-1])['frames']; print('f32', d['value']/1e9, d['roofline']['frac'], 'f64', d['f64_scores']['value']/1e9, d['f64_scores']['frac'])"
bash tools/pmc.sh r04cos --no-search --no-precomputed --no-stream --no-ingest --no-frames-f64 > $O/cos_pmc.log 2>&1
python3 -c "
import json; d=json.loads(open('gpurun_out/pmc_r04cos/summary.txt').read()); print({k: v.get('hbm_bytes_per_launch') for k, v in d.items()})"
