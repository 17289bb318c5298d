#!/usr/bin/env python3
"""Summarise a tools/gpu_ab_kernels.sh run: per-kernel average µs (rocprofv3 kernel stats) for the
baseline and candidate rounds, engine kernel time, tree identity, test tail and the bench line.
Usage: python tools/ab_summary.py gpurun_out/<name>"""
import csv
import json
import os
import sys

d = sys.argv[1]
rows = {}
for arm in ("base", "cand"):
    for r in (1, 2, 3):
        p = os.path.join(d, f"{arm}_{r}", "k_kernel_stats.csv")
        if not os.path.exists(p):
            continue
        for row in csv.DictReader(open(p)):
            k = row["Name"].split("(")[0].replace("void nm03::gpu::", "")
            rows.setdefault(k, {}).setdefault(arm, []).append(float(row["AverageNs"]) / 1e3)
        t = open(os.path.join(d, f"{arm}_{r}.log")).read()
        j = json.loads(t[t.index('{"config"'):].splitlines()[0])
        rows.setdefault("engine kernels_s (ms / 5 steps)", {}).setdefault(arm, []).append(j["kernels_s"] * 1e3)
print(f"{'kernel':45s} {'baseline':>26s} {'candidate':>26s}")
for k, v in rows.items():
    f = lambda a: " ".join(f"{x:7.2f}" for x in v.get(a, []))
    print(f"{k[:45]:45s} {f('base'):>26s} {f('cand'):>26s}")
print("trees:", open(os.path.join(d, "diff_ok.txt")).read().strip() if os.path.exists(os.path.join(d, "diff_ok.txt")) else "DIFFER")
print("tests:", open(os.path.join(d, "pytest_gpu.log")).read().strip().splitlines()[-1])
b = os.path.join(d, "bench.json")
if os.path.exists(b):
    j = json.load(open(b))
    print("bench:", j["value"], "slices/s", j["ms_per_step"], "ms/step")
    p = os.path.join(d, "bench", "k_kernel_stats.csv")
    if os.path.exists(p):
        for row in csv.DictReader(open(p)):
            print(f"  bench {row['Name'].split('(')[0][:50]:50s} {float(row['AverageNs'])/1e3:7.1f} us x {row['Calls']}")
