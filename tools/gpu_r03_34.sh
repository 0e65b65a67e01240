#!/bin/bash
# N = 2 rehearsal of the bench's multi-rank path on one GPU (gloo collectives, both ranks on device 0)
export TMPDIR=/tmp
HQ_BENCH_SAME_DEVICE=1 HQ_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r03_n2b.json 2> gpurun_out/r03_n2b.err
rc=$?; echo "n2 rc=$rc"; tail -3 gpurun_out/r03_n2b.err
python3 -c "
import json; d=json.loads(open('gpurun_out/r03_n2b.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,1), 'search', round(d['search']['value']/1e6,3), 'frames', round(d['frames']['value']/1e9,2), 'stream', round(d['stream']['value'],1), 'precomp', round(d['precomputed']['value']/1e6,1))
"
exit $rc
