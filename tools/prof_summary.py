#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --kernel-trace --stats directory (kernel_stats.csv)."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    fs = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    if not fs:
        print(d, "no kernel_stats.csv")
        continue
    print("==", d)
    for x in list(csv.DictReader(open(fs[0])))[:16]:
        print(x["Name"][:70].ljust(70), x["Calls"].rjust(5), f'{float(x["AverageNs"]) / 1e3:9.1f} us',
              f'{float(x["TotalDurationNs"]) / 1e3:10.0f} us total')
