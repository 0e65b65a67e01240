#!/bin/bash
# PMC passes (SQ counters) for one kernel of a command.  usage: tools/pmc_kernel.sh <kernel-substring> <cmd...>
set -u
KN=$1; shift
OUT=gpurun_out/pmc_$KN
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P3="SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; }
done
python3 - "$KN" <<'PY'
import csv, glob, sys
from collections import defaultdict
kn = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_{kn}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kn in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {c: sum(x) / len(x) for c, x in vals.items()}
w = avg.get("SQ_WAVES", 1)
print("per wave", {c: round(x / w, 1) for c, x in sorted(avg.items())})
PY
