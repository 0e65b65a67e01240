#!/bin/bash
# PMC counters of the level-0 scan kernels for two variants (default, score-only).
set -u
OUT=gpurun_out/pmc_scan
mkdir -p $OUT
export TMPDIR=/tmp
for v in default score-only; do
  SCAN_EXPT_ONLY=$v timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/$v -o $v --output-format csv -- python tools/scan_expt.py > $OUT/$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for v in ("default", "score-only"):
    vals = defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_scan/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_scan0f" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {c: sum(x) / len(x) for c, x in vals.items()}
    w = avg.get("SQ_WAVES", 1)
    print(v, {c: round(x / w, 1) for c, x in sorted(avg.items())})
PY
