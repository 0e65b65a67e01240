#!/bin/bash
# cfg5 chunk kernel A/B: chunks per wave 2 (default) / 4 (128-B aligned frame runs), non-temporal stores
export TMPDIR=/tmp
for o in; do
  opts=""; if [ "$o" != "-" ]; then for x in ${o//,/ }; do opts="$opts --option $x"; done; fi
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-search --no-precomputed --no-ingest --no-frames --stream-steps 10 $opts > gpurun_out/r03_c25.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_c25.json'))['stream']; print('$o', round(d['value'],1), 'GB/s', round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],3), 'ms')"
done
# S7 skeleton costs (diagnostics build, wrong scores): 90 no stores, 91 no MFMAs, 92 no K-loop barriers
DIAG=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
for k in 0 91 93 94 95 0; do
  HQ_LIB_VARIANT=$DIAG HQ_COS_KERNEL=$k timeout -k 10 120 python bench.py --no-search --no-stream --no-precomputed --no-ingest --no-cpu --steps 2 > gpurun_out/r03_f25.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03_f25.json'))['frames']; print('cos diag $k', round(d['value']/1e9,2), round(d['roofline']['frac'],3), round(d['ms_per_step'],3))"
done
