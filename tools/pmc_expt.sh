#!/bin/bash
# P1/P2 PMC passes of k_scan0g under the diagnostics build's timing experiments (HQ_SCAN_EXPT 0 / 6)
export TMPDIR=/tmp
export HQ_LIB_VARIANT=$PWD/hilbert-quantization_amd/hq_mi355x/libhq_mi355x_diag.so
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_EXP"
for e in 0 6; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    HQ_SCAN_EXPT=$e HQ_SCAN_WPB=1 timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmcx_$e/p$i -o p$i --output-format csv -- python3 tools/scan_debug.py > gpurun_out/pmcx_${e}_p$i.log 2>&1 || { echo "expt $e pass $i failed"; tail -3 gpurun_out/pmcx_${e}_p$i.log; }
  done
  python3 - "$e" <<'PY'
import csv, glob, sys
from collections import defaultdict
e = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmcx_{e}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_scan0g" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {c: sum(x) / len(x) for c, x in vals.items()}
w = avg.get("SQ_WAVES", 1)
print("expt", e, "per wave", {c: round(x / w, 1) for c, x in sorted(avg.items())})
PY
done
