#!/usr/bin/env python3
"""Per-step timeline breakdown of a rocprofv3 run of bench.py.

Run (on the GPU box, no counters):
  NM03_ROCTX=1 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv \
      -d gpurun_out/tl -o bench -- python3 bench.py --steps 3 --warmup 1
then `python tools/timeline.py gpurun_out/tl` (per step, `--no-pipeline` runs), or
`--window` for the pipelined default: utilisation over the whole `bench.steps` range.

bench.py pushes a `bench.step` roctx range around every engine run when NM03_ROCTX is set; the
engine pushes `nm03.load` (per slice), `nm03.gpu_batch` (per batch) and `nm03.export` (per slice).
For each step the report gives the union-busy time of kernels, H2D copies, host loads and host
exports, the GPU idle time (no kernel and no copy), and the fill (step start → first H2D) and
drain (last kernel → step end) latencies.
"""
import csv
import glob
import os
import sys


def _rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    return hits[0] if hits else None


def union(iv, lo=None, hi=None):
    """Total length of the union of intervals, optionally clipped to [lo, hi]."""
    segs = []
    for a, b in iv:
        if lo is not None:
            a, b = max(a, lo), min(b, hi)
        if b > a:
            segs.append((a, b))
    segs.sort()
    tot, cur_a, cur_b = 0, None, None
    for a, b in segs:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def load(d):
    ev = {"kernel": [], "h2d": [], "d2h": [], "marker": []}
    kp = _find(d, "kernel_trace.csv")
    if kp:
        for r in _rows(kp):
            ev["kernel"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    mp = _find(d, "memory_copy_trace.csv")
    if mp:
        for r in _rows(mp):
            direction = (r.get("Direction") or r.get("Operation") or "").upper()
            key = "h2d" if "HOST_TO_DEVICE" in direction else "d2h" if "DEVICE_TO_HOST" in direction else None
            if key:
                ev[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), direction))
    ap = _find(d, "marker_api_trace.csv")
    if ap:
        for r in _rows(ap):
            name = r.get("Function") or r.get("Name") or ""
            msg = r.get("Message") or r.get("Name") or name
            ev["marker"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), msg))
    return ev


def window(d):
    """Pipelined bench (overlapping passes): utilisation over the whole `bench.steps` range — union-busy
    fractions of kernels, H2D copies and either, mean kernel concurrency, per-kernel totals."""
    ev = load(d)
    rng = [(a, b) for a, b, m in ev["marker"] if "bench.steps" in m]
    if rng:
        lo, hi = rng[-1]
    else:  # no roctx: the middle 80% of the kernels' span (leaves warm-up and tear-down out)
        allv = [x for k in ("kernel", "h2d") for x in ev[k]]
        lo, hi = min(a for a, _, _ in allv), max(b for _, b, _ in allv)
        lo, hi = lo + (hi - lo) // 10, hi - (hi - lo) // 10
    span = hi - lo
    k = [(a, b) for a, b, _ in ev["kernel"]]
    h = [(a, b) for a, b, _ in ev["h2d"]]
    dh = [(a, b) for a, b, _ in ev["d2h"]]
    ksum = sum(min(b, hi) - max(a, lo) for a, b in k if b > lo and a < hi)
    print(f"window {span / 1e6:.2f} ms")
    for name, iv in (("kernels", k), ("h2d", h), ("d2h", dh), ("kernels|h2d", k + h)):
        u = union(iv, lo, hi)
        print(f"  {name:12s} busy {u / 1e6:9.2f} ms  {100.0 * u / span:5.1f}% of the window")
    ku = union(k, lo, hi)
    if ku:
        print(f"  mean kernels in flight while any runs: {ksum / ku:.2f}")
    tot = {}
    for a, b, n in ev["kernel"]:
        if b > lo and a < hi:
            t = tot.setdefault(n, [0, 0])
            t[0] += min(b, hi) - max(a, lo)
            t[1] += 1
    for n, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0]):
        print(f"  {t / 1e6:9.2f} ms {100.0 * t / span:5.1f}%  n={c:6d}  mean {t / c / 1e3:7.1f} us  {n[:70]}")
    if h:
        durs = sorted((b - a) / 1e3 for a, b in h if b > lo and a < hi)
        if durs:
            print(f"  h2d copies: n={len(durs)} median={durs[len(durs) // 2]:.1f}us max={durs[-1]:.1f}us")


def report(d):
    ev = load(d)
    steps = sorted((a, b) for a, b, m in ev["marker"] if "bench.step" in m and "bench.steps" not in m)
    if not steps:  # fall back to the whole trace as one step
        allv = [x for k in ("kernel", "h2d") for x in ev[k]]
        steps = [(min(a for a, _, _ in allv), max(b for _, b, _ in allv))]
    us = 1e-3
    print(f"{'step':>4} {'wall':>8} {'kern':>8} {'h2d':>8} {'gpu_busy':>8} {'gpu_idle':>8} {'load':>8} {'export':>8}"
          f" {'fill':>7} {'drain':>7}   (us)")
    for i, (lo, hi) in enumerate(steps):
        k = [(a, b) for a, b, _ in ev["kernel"]]
        h = [(a, b) for a, b, _ in ev["h2d"]]
        ld = [(a, b) for a, b, m in ev["marker"] if "nm03.load" in m]
        ex = [(a, b) for a, b, m in ev["marker"] if "nm03.export" in m]
        busy = union(k + h, lo, hi)
        first_h2d = min((a for a, _ in h if lo <= a <= hi), default=lo)
        last_k = max((b for _, b in k if lo <= b <= hi), default=hi)
        print(f"{i:>4} {(hi - lo) * us:8.0f} {union(k, lo, hi) * us:8.0f} {union(h, lo, hi) * us:8.0f}"
              f" {busy * us:8.0f} {(hi - lo - busy) * us:8.0f} {union(ld, lo, hi) * us:8.0f}"
              f" {union(ex, lo, hi) * us:8.0f} {(first_h2d - lo) * us:7.0f} {(hi - last_k) * us:7.0f}")
    # H2D bandwidth estimate per copy (bytes are not in the trace: report durations)
    if ev["h2d"]:
        durs = sorted((b - a) * us for a, b, _ in ev["h2d"])
        print(f"h2d copies: n={len(durs)} median={durs[len(durs) // 2]:.0f}us max={durs[-1]:.0f}us")
    if len(steps) and "-v" in sys.argv:
        lo, hi = steps[-1]
        rows = []
        for kind in ("kernel", "h2d", "d2h"):
            rows += [(a, b, kind, n) for a, b, n in ev[kind] if lo <= a <= hi]
        rows += [(a, b, "marker", n) for a, b, n in ev["marker"] if lo <= a <= hi and "gpu_batch" in n]
        for a, b, kind, n in sorted(rows):
            print(f"  {(a - lo) * us:8.1f} +{(b - a) * us:7.1f} {kind:7s} {n[:60]}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("-")]
    (window if "--window" in sys.argv else report)(args[0] if args else "gpurun_out/tl")
