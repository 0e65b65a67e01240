#!/usr/bin/env python3
"""GPU idle time between kernels in a rocprofv3 --kernel-trace directory: over the last n steps (a step
starts at each dispatch of <anchor>, a kernel-name substring; with <stop>, only dispatches before the
first <stop> dispatch count), the busy time per kernel and the gap time between consecutive dispatches.
usage: trace_gaps.py <dir> <anchor> [n] [stop]"""
import csv
import glob
import sys
from collections import defaultdict

d, anchor = sys.argv[1], sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 10
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 4:
    cut = next((i for i, r in enumerate(rows) if sys.argv[4] in r["Kernel_Name"]), len(rows))
    rows = rows[:cut]
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
if len(starts) < last + 1:
    sys.exit(f"only {len(starts)} anchors")
seg = rows[starts[-last - 1]:starts[-1]]
busy = defaultdict(float)
gaps = 0.0
gap_after = defaultdict(float)
for a, b in zip(seg, seg[1:] + [rows[starts[-1]]]):
    t0, t1 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    busy[a["Kernel_Name"][:60]] += (t1 - t0) / last / 1e3
    g = max(0, int(b["Start_Timestamp"]) - t1) / last / 1e3
    gaps += g
    gap_after[a["Kernel_Name"][:60]] += g
span = (int(rows[starts[-1]]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / last / 1e3
print(f"per step: span {span:.1f} us, kernels {len(seg) / last:.1f}, busy {sum(busy.values()):.1f} us, gaps {gaps:.1f} us")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {k.ljust(60)} {v:7.1f} us   gap after {gap_after[k]:6.1f} us")
