#!/bin/bash
# k_scan0f time under diagnostic knobs (HQ_SCAN_EXPT): 0 default, 7 no full filter / inserts,
# Needs the diagnostics build (make -C hilbert-quantization_amd/csrc DIAG=1): the default build compiles HQ_SCAN_EXPT away.
# 8 pre-filter never fires (results wrong; timing only)
for e in ${EXPTS:-0 7 8}; do
  HQ_SCAN_EXPT=$e bash tools/search_only_prof.sh e$e > /dev/null 2>&1
  python3 - gpurun_out/sprof_e$e <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    if 'k_scan0f' in x['Name']: print(sys.argv[1], x["Name"][:30], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us")
PY
done
