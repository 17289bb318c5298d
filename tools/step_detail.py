#!/usr/bin/env python3
"""Event list of one bench step from a rocprofv3 timeline run (tools/gpu_timeline.sh): GPU batches,
uploads, kernels, plus per-slot load/export windows. Usage: python tools/step_detail.py <dir> [step]"""
import csv
import glob
import statistics
import sys


def rows(d, suffix):
    return list(csv.DictReader(open(glob.glob(d + '/**/*' + suffix, recursive=True)[0])))


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    mk, kt, mc = rows(d, 'marker_api_trace.csv'), rows(d, 'kernel_trace.csv'), rows(d, 'memory_copy_trace.csv')
    steps = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in mk if r['Function'] == 'bench.step')
    a, b = steps[k]
    ev = []
    for r in mk:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if a <= s <= b and r['Function'] != 'bench.step':
            ev.append((s, e, r['Function'], r['Thread_Id']))
    for r in kt:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if a <= s <= b:
            ev.append((s, e, 'K ' + r['Kernel_Name'].split('(')[0].split('::')[-1][:24], ''))
    for r in mc:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if a <= s <= b:
            ev.append((s, e, 'H2D', ''))
    ev.sort()
    loads = [x for x in ev if x[2] == 'nm03.load']
    exps = [x for x in ev if x[2] == 'nm03.export']
    print('step %.1f us; loads %d exports %d; load median %.1f us, export median %.1f us' % (
        (b - a) / 1e3, len(loads), len(exps), statistics.median([(x[1] - x[0]) / 1e3 for x in loads]),
        statistics.median([(x[1] - x[0]) / 1e3 for x in exps])))
    h2d = sorted((x[0], x[1]) for x in ev if x[2] == 'H2D')
    gaps, cur = [], None
    for s, e in h2d:
        if cur is not None and s > cur:
            gaps.append(((cur - a) / 1e3, (s - cur) / 1e3))
        cur = e if cur is None else max(cur, e)
    print('H2D first %.1f last end %.1f; gaps >10us: %s' % ((h2d[0][0] - a) / 1e3, (cur - a) / 1e3,
                                                           [(round(g[0]), round(g[1])) for g in gaps if g[1] > 10]))
    for s, e, n, t in ev:
        if n in ('nm03.load', 'nm03.export', 'H2D'):
            continue
        print('%8.1f +%7.1f %s %s' % ((s - a) / 1e3, (e - s) / 1e3, n, t))
    print('last load end %.1f, last export end %.1f' % ((max(x[1] for x in loads) - a) / 1e3,
                                                      (max(x[1] for x in exps) - a) / 1e3))


if __name__ == '__main__':
    main()
