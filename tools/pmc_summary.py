#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel (sum over dispatches)."""
import collections
import csv
import glob
import os
import sys


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        for r in csv.DictReader(open(path, newline="")):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nm03::gpu::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (path, r.get("Dispatch_Id"))
            if did not in seen:
                seen.add(did)
                calls[(k, path)] += 1
    for k, c in sorted(agg.items()):
        print(k)
        waves = c.get("SQ_WAVES", 0)
        for name, v in sorted(c.items()):
            extra = f"   per-wave {v / waves:10.1f}" if waves and name.startswith("SQ_INSTS") else ""
            print(f"   {name:24s} {v:16.0f}{extra}")
        if c.get("SQ_WAVE_CYCLES") and c.get("SQ_ACTIVE_INST_VALU"):
            print(f"   VALU active / wave-cycles = {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
