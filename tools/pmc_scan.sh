#!/bin/bash
# PMC counters of the f32 level-0 scan kernel (tools/scan_expt.py, default variant), two passes.
set -u
OUT=gpurun_out/pmc_scan
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_IFETCH SQ_ACTIVE_INST_VALU"
P2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python ${SCAN_SCRIPT:-tools/scan_debug.py} > $OUT/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob("gpurun_out/pmc_scan/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_scan0f" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {c: sum(x) / len(x) for c, x in vals.items()}
w = avg.get("SQ_WAVES", 1)
print({c: round(x, 1) for c, x in sorted(avg.items())})
print("per wave", {c: round(x / w, 1) for c, x in sorted(avg.items())})
PY
