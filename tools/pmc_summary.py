#!/usr/bin/env python3
"""Summarise tools/gpu_pmc_jpeg.sh output: per-wave SQ counters of the JPEG encoder per truncation
variant, and of every kernel in the full pipeline (variant 0). VALU-active / wave-cycles × resident
waves per SIMD (4 for the encoder) approximates how busy the SIMDs' VALUs are.
Usage: python tools/pmc_summary.py gpurun_out/<name>"""
import collections
import csv
import os
import sys

d = sys.argv[1]
names = {7: "tables + ticket", 1: "+ render / staging", 16: "+ FDCT + quantisation", 2: "+ AC coding",
         4: "+ DC, scan, bit range, look-back", 0: "full encoder", 40: "gray images only", 41: "label images only"}
print("JPEG encoder, per-wave averages over all dispatches (isolated engine runs, 1 stream, batch 96)")
print(f"{'variant':40s} {'VALU':>6} {'SALU':>6} {'LDS':>5} {'wave-cyc':>9} {'VALU/wc':>8} {'wait/wc':>8}")
full = {}
for v in (7, 1, 16, 2, 4, 0, 40, 41):
    p = os.path.join(d, f"v{v}", "k_counter_collection.csv")
    if not os.path.exists(p):
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void nm03::gpu::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, c in acc.items():
        w = c["SQ_WAVES"]
        if "jpeg" in k and w:
            print(f"jpeg={v:<3} {names[v]:32s} {c['SQ_INSTS_VALU']/w:6.0f} {c['SQ_INSTS_SALU']/w:6.0f} "
                  f"{c['SQ_INSTS_LDS']/w:5.0f} {c['SQ_WAVE_CYCLES']/w:9.0f} "
                  f"{c['SQ_ACTIVE_INST_VALU']/c['SQ_WAVE_CYCLES']:8.3f} {c['SQ_WAIT_INST_ANY']/c['SQ_WAVE_CYCLES']:8.3f}")
        if v == 0:
            full[k] = (len(disp[k]), c)
print("\nEvery kernel of the full pipeline (variant 0):")
for k, (n, c) in full.items():
    w = c["SQ_WAVES"]
    if not w:
        continue
    print(f"{k[:40]:40s} waves/dispatch {w/n:7.0f}  VALU/wave {c['SQ_INSTS_VALU']/w:6.0f}  SALU/wave {c['SQ_INSTS_SALU']/w:5.0f}  "
          f"VALU/wc {c['SQ_ACTIVE_INST_VALU']/c['SQ_WAVE_CYCLES']:.3f}  wait/wc {c['SQ_WAIT_INST_ANY']/c['SQ_WAVE_CYCLES']:.3f}")
