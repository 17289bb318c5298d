#!/usr/bin/env python3
"""Median duration of every kernel's full-size dispatches (the largest grid it ran with) from rocprofv3
--kernel-trace CSVs, one line per file: what profiles/r5/flags/ and profiles/r5/huff/ quote.
Usage: python tools/kernel_medians.py <dir>/*_kernel_trace.csv"""
import collections
import csv
import statistics
import sys

for f in sys.argv[1:]:
    runs = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nm03::gpu::", "")
        if "rocclr" in k or "__amd" in k:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        runs[k].append((grid, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["VGPR_Count"]))
    parts = []
    for k, v in sorted(runs.items()):
        g = max(x[0] for x in v)
        full = [x[1] for x in v if x[0] == g]
        parts.append(f"{k.split('<')[0][:12]:12s} {statistics.median(full):6.1f} us (n={len(full)}, vgpr={v[0][2]})")
    print(f"{f}:\n  " + "\n  ".join(parts))
