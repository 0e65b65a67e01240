#!/bin/bash
# LDS / issue PMC passes on one bench section (no tracing domains): instruction mix, LDS bank
# conflicts and waits per kernel.  usage: tools/pmc_lds.sh <tag> <bench args...>
set -u
TAG=${1:-lds}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py --steps 2 --warmup 0 --no-cpu "${BENCH_ARGS[@]}" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
BENCH_ARGS=("$@")
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
python3 tools/pmc_traffic.py $OUT > $OUT/summary.txt 2>&1
exit 0
