#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output: the SQ counters of every kernel, summed over the run's
dispatches across the per-group passes (gpurun_out/pmc/p*/run_counter_collection.csv), as per-wave
instruction counts and per-wave-cycle activity. VALU-active / wave-cycles × resident waves per SIMD
approximates how busy the SIMDs' VALUs are.
Usage: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for p in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void nm03::gpu::", "")
        if "rocclr" in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':40s} {'waves':>8} {'VALU/w':>7} {'SALU/w':>7} {'LDS/w':>6} {'VALU/wc':>8} {'wait/wc':>8} "
      f"{'LDSbc/LDSact':>12} {'VMEMrd/w':>8} {'VMEMwr/w':>8}")
for k, c in sorted(acc.items()):
    w = c.get("SQ_WAVES", 0.0) or 1.0
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    lds_act = c.get("SQ_ACTIVE_INST_LDS", 0.0) or 1.0
    print(f"{k[:40]:40s} {w:8.0f} {c.get('SQ_INSTS_VALU', 0) / w:7.0f} {c.get('SQ_INSTS_SALU', 0) / w:7.0f} "
          f"{c.get('SQ_INSTS_LDS', 0) / w:6.0f} {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:8.3f} "
          f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:8.3f} {c.get('SQ_LDS_BANK_CONFLICT', 0) / lds_act:12.3f} "
          f"{c.get('SQ_INSTS_VMEM_RD', 0) / w:8.1f} {c.get('SQ_INSTS_VMEM_WR', 0) / w:8.1f}")
