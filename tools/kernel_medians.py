#!/usr/bin/env python3
"""Median duration of every kernel's full-size dispatches (the largest grid it ran with) from rocprofv3
--kernel-trace CSVs, one line per file: what profiles/r5/flags/ and profiles/r5/huff/ quote.
Usage: python tools/kernel_medians.py <dir>/*_kernel_trace.csv
       python tools/kernel_medians.py --summary gpurun_out/<name>/summary.txt   (gpu_kmedians.sh: medians
       and ranges per variant over the rounds)"""
import collections
import csv
import re
import statistics
import sys

if sys.argv[1:2] == ["--summary"]:
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    v = None
    for line in open(sys.argv[2]):
        m = re.match(r"== variant \d+ \((.*)\) round \d+: (.*)", line)
        if m:
            v = m.group(1)
            t = re.search(r"(\d+)$", m.group(2))
            if t:
                d[v]["slices/s"].append(int(t.group(1)))
            continue
        m = re.match(r"\s+(\S+)\s+([\d.]+) us", line)
        if m and v:
            d[v][m.group(1)].append(float(m.group(2)))
    for v, ks in d.items():
        print(f"{v:28s} " + "  ".join(f"{k} {statistics.median(x):.1f} [{min(x):.1f}-{max(x):.1f}]"
                                      for k, x in ks.items() if not k.startswith("build_norm")))
    sys.exit(0)

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
