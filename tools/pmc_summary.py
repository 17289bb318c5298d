#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel (sum over dispatches).

    pmc_summary.py <pmc dir> [kernel_stats.csv]

With a kernel_stats.csv from a --kernel-trace --stats run of the same workload, derived rates are
printed too: HBM/L2 bytes per dispatch and achieved bandwidth (FETCH_SIZE / WRITE_SIZE are in KiB),
VALU and LDS activity per wave-cycle, and LDS bank-conflict cycles per LDS instruction.
"""
import collections
import csv
import glob
import os
import sys


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("nm03::gpu::", "")


def load_stats(path):
    out = {}
    if path and os.path.exists(path):
        for r in csv.DictReader(open(path, newline="")):
            out[_short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    return out


def main(d, stats_path=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(path, newline="")):
            k = _short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add((path, r.get("Dispatch_Id")))
    stats = load_stats(stats_path)
    for k, c in sorted(agg.items()):
        print(k)
        waves = c.get("SQ_WAVES", 0)
        for name, v in sorted(c.items()):
            extra = f"   per-wave {v / waves:10.1f}" if waves and name.startswith("SQ_INSTS") else ""
            print(f"   {name:24s} {v:16.0f}{extra}")
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            if c.get("SQ_ACTIVE_INST_VALU"):
                print(f"   VALU active / wave-cycles = {c['SQ_ACTIVE_INST_VALU'] / wc:.3f}")
            if c.get("SQ_ACTIVE_INST_LDS"):
                print(f"   LDS active / wave-cycles  = {c['SQ_ACTIVE_INST_LDS'] / wc:.3f}")
            if c.get("SQ_WAIT_INST_ANY"):
                print(f"   waiting / wave-cycles     = {c['SQ_WAIT_INST_ANY'] / wc:.3f}")
        if c.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
            print(f"   LDS bank-conflict cycles per LDS inst = {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.3f}")
        st = stats.get(k)
        for cn, label in (("FETCH_SIZE", "read"), ("WRITE_SIZE", "written")):
            if cn in c and disp[k][cn]:
                per = c[cn] * 1024.0 / len(disp[k][cn])
                line = f"   bytes {label} per dispatch = {per / 1e6:8.3f} MB"
                if st:
                    line += f"   -> {per / st[1]:7.1f} GB/s at the isolated {st[1] / 1e3:.1f} us"
                print(line)
        if st:
            print(f"   isolated duration: {st[1] / 1e3:.1f} us avg over {st[0]} calls")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc", sys.argv[2] if len(sys.argv) > 2 else None)
