#!/bin/bash
# Phase costs of the pre-computed index kernel (HQ_PRECOMP_DIAG bits skip phases: 1 small squares,
# 2 leaves, 4 load/scatter, 8 stores; wrong averages, timing only) on a DIAG variant library.
# Build the variant first (then rebuild the normal library):
#   make -C hilbert-quantization_amd/csrc clean && make -C hilbert-quantization_amd/csrc DIAG=1 OUT=$PWD/diag_variant.so
#   make -C hilbert-quantization_amd/csrc clean && make -C hilbert-quantization_amd/csrc
for v in "HQ_PRECOMP_SKIP=0" "HQ_PRECOMP_SKIP=0 HQ_PRECOMP_DIAG=15" "HQ_NONE=1" "HQ_PRECOMP_DIAG=1" "HQ_PRECOMP_DIAG=2" "HQ_PRECOMP_DIAG=4" "HQ_PRECOMP_DIAG=8" "HQ_PRECOMP_DIAG=15" "HQ_PRECOMP_DIAG=7" "HQ_PRECOMP_DIAG=3"; do
  r=$(env HQ_LIB_VARIANT=$PWD/diag_variant.so HQ_PRECOMP_GRID=16384 $v timeout -k 10 120 python bench.py --no-search --no-stream --no-cpu --no-ingest --no-frames --steps 8 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['precomputed']; print(round(d['value']/1e6,1), round(d['ms_per_step'],3))") || exit 1
  echo "$v: $r"
done
