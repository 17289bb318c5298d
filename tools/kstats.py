#!/usr/bin/env python3
"""Summarise a rocprofv3 *_kernel_stats.csv: python tools/kstats.py gpurun_out/prof_iter/bench_kernel_stats.csv"""
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== {f}: {tot/1e6:.3f} ms total kernel time")
    for r in rows:
        name = r["Name"].split("(")[0].replace("nm03::gpu::", "").replace("void ", "")
        print(f"  {name:34s} calls={int(r['Calls']):5d} total={float(r['TotalDurationNs'])/1e6:8.3f} ms "
              f"avg={float(r['AverageNs'])/1e3:8.2f} us  {float(r['Percentage']):5.1f}%")
