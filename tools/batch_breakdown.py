#!/usr/bin/env python3
"""Per-batch kernel breakdown of the progressive search legs in a rocprofv3 --kernel-trace directory: batches
are the kernel sequences between two query preparations (k_seg_prepare_pack0); sequences of the same kernel
pattern are grouped, and each group's median batch span, busy time and per-kernel times are printed (groups
with a long scan are the 8M-row cfg4 leg).  usage: batch_breakdown.py <dir> [min_batches]"""
import csv
import glob
import statistics as S
import sys
from collections import defaultdict

d = sys.argv[1]
minb = int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_seg_prepare_pack0" in r["Kernel_Name"]]
groups = defaultdict(list)
for a, b in zip(idx, idx[1:]):
    seg = rows[a:b]
    key = tuple(r["Kernel_Name"].split("(")[0][-28:] for r in seg)
    scan = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg if "scan0g" in r["Kernel_Name"]]
    cls = "long-scan" if scan and scan[0] > 400_000 else "scan<400us"
    groups[(cls, key)].append((a, b))
for (cls, key), segs in sorted(groups.items(), key=lambda x: -len(x[1])):
    if len(segs) < minb:
        continue
    spans, busy = [], []
    per = defaultdict(list)
    for a, b in segs:
        seg = rows[a:b]
        spans.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
        busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3)
        for r in seg:
            per[r["Kernel_Name"].split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{cls}: {len(segs)} batches, median span {S.median(spans):.1f} us, busy {S.median(busy):.1f} us")
    for k, v in sorted(per.items(), key=lambda x: -S.median(x[1])):
        print(f"    {k:40s} {S.median(v):8.1f} us")
