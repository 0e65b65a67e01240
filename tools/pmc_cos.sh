#!/bin/bash
# PMC passes on the S7 frames bench only (k_cos_* kernels): MFMA busy, LDS instructions / conflicts / waits.
# usage: tools/pmc_cos.sh <tag> [env assignments...]
set -u
TAG=${1:-cos}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do export "$v"; done
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu --no-search --no-stream --no-precomputed --no-ingest > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM && \
run fetch FETCH_SIZE TCC_HIT_sum && run write WRITE_SIZE
python3 tools/pmc_traffic.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
exit 0
