#!/bin/bash
# PMC passes for the level-0 scan kernel on the bench corpus (tools/scan_debug.py): issue/wait
# counters, instruction mix and L2 hit / memory-side read requests.
set -u
OUT=gpurun_out/pmc_scan2
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 tools/scan_debug.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob("gpurun_out/pmc_scan2/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_scan0f" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {c: sum(x) / len(x) for c, x in vals.items()}
w = avg.get("SQ_WAVES", 1)
print("total", {c: round(x, 1) for c, x in sorted(avg.items())})
print("per wave", {c: round(x / w, 1) for c, x in sorted(avg.items())})
PY
