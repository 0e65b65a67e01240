#!/bin/bash
# N = 2 and N = 4 rehearsals of the CURRENT bench's multi-rank path on one GPU (gloo collectives, every rank
# on device 0: RCCL refuses two ranks on one GPU) — the driver's round-end scaling runs take this path with RCCL
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for n in 2 4; do
HQ_BENCH_SAME_DEVICE=1 HQ_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $n --steps 5 --warmup 2 --no-cpu > $O/r06_n${n}.json 2> $O/r06_n${n}.err
rc=$?; echo "n$n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/r06_n${n}.err; exit $rc; }
N=$n python3 -c "
import json, os; d=json.loads(open(os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/r06_n' + os.environ['N'] + '.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,1), json.dumps(d.get('summary')))
"
done
