#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no tracing domains) on a short bench run.
# usage: tools/pmc.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu "${BENCH_ARGS[@]}" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
BENCH_ARGS=("$@")
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS && \
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH
python3 tools/pmc_traffic.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
exit 0
