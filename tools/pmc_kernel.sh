#!/bin/bash
# PMC passes (one rocprofv3 run per pass) for one kernel of tools/scan_debug.py:
#   tools/pmc_kernel.sh <kernel-name-substring> <outdir> [level0|overall|chunk]
# P1 issue/wait split, P2 instruction mix + MFMA busy, P3 L2 hits/misses + clock, P4 LDS + L1.
set -u
K=${1:-k_scan0g}
OUT=${2:-gpurun_out/pmc_$K}
MODE=${3:-level0}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
P4="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  DRV="tools/scan_debug.py $MODE"
  [ "$MODE" = "chunk" ] && DRV="tools/chunk_debug.py"
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 $DRV > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - "$K" "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
k, out = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {c: sum(x) / len(x) for c, x in vals.items()}
w = avg.get("SQ_WAVES", 1)
print("kernel", k, "launches", {c: len(x) for c, x in vals.items()}.get("SQ_WAVES"))
print("total", {c: round(x, 1) for c, x in sorted(avg.items())})
print("per wave", {c: round(x / w, 1) for c, x in sorted(avg.items())})
wc = avg.get("SQ_WAVE_CYCLES")
if wc:
    print("fractions of SQ_WAVE_CYCLES", {c: round(avg[c] / wc, 3) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS") if c in avg})
PY
