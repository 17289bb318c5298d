#!/usr/bin/env python3
"""Single-pass latency breakdown from a rocprofv3 trace of bench.py (tools/gpu_r3_hiptrace.sh):
for each bench.step with the given number of loads, per slot thread: loads, HIP calls (memcpy,
launches, event records, queries), copies and kernels relative to the step start.

    tl_single.py <trace dir> [n_loads=58] [max_steps=2]
"""
import collections
import csv
import glob
import sys


def rows(d, suffix):
    p = glob.glob(f"{d}/**/*{suffix}", recursive=True)
    return list(csv.DictReader(open(p[0]))) if p else []


def main(d, nload=58, maxs=2):
    mk, kt, mc, api = (rows(d, s) for s in ("marker_api_trace.csv", "kernel_trace.csv", "memory_copy_trace.csv",
                                              "hip_api_trace.csv"))
    steps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in mk if r["Function"] == "bench.step")
    shown = 0
    for s0, s1 in steps:
        inside = lambda r: s0 <= int(r["Start_Timestamp"]) <= s1
        loads = [r for r in mk if r["Function"] == "nm03.load" and inside(r)]
        if len(loads) != nload:
            continue
        f = lambda x: (int(x) - s0) / 1e3
        print(f"== step wall {(s1 - s0) / 1e3:.0f} us")
        ev = []
        for r in mk:
            if inside(r) and r["Function"] not in ("bench.step",):
                ev.append((f(r["Start_Timestamp"]), f(r["End_Timestamp"]), r["Function"], "T" + r["Thread_Id"]))
        for r in api:
            if inside(r) and r["Function"] in ("hipMemcpyAsync", "hipLaunchKernel", "hipExtLaunchKernel", "hipEventRecord",
                                                "hipModuleLaunchKernel", "hipGraphLaunch"):
                ev.append((f(r["Start_Timestamp"]), f(r["End_Timestamp"]), r["Function"], "T" + r["Thread_Id"]))
        for r in kt:
            if inside(r):
                ev.append((f(r["Start_Timestamp"]), f(r["End_Timestamp"]), "K " + r["Kernel_Name"].split("(")[0][16:40],
                           "S" + r["Stream_Id"]))
        for r in mc:
            if inside(r):
                ev.append((f(r["Start_Timestamp"]), f(r["End_Timestamp"]), "COPY " + r["Direction"][:6], "S" + r["Stream_Id"]))
        q = collections.Counter(r["Thread_Id"] for r in api if inside(r) and r["Function"] == "hipEventQuery")
        ev.sort()
        agg = collections.defaultdict(list)
        for a, b, n, t in ev:
            if n in ("nm03.load", "nm03.export"):
                agg[n].append((a, b))
                continue
            print(f"  {a:8.1f} +{b - a:7.1f}  {n:32s} {t}")
        for n, v in agg.items():
            ends = sorted(b for a, b in v)
            print(f"  {n}: {len(v)} first {min(a for a, b in v):.1f} ends q0..q4 {[round(ends[int(k * (len(ends) - 1) / 4)], 1) for k in range(5)]}"
                  f" mean dur {sum(b - a for a, b in v) / len(v):.1f}")
        print("  hipEventQuery calls per thread:", dict(q))
        shown += 1
        if shown >= maxs:
            break


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
