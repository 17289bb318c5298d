#!/usr/bin/env python3
"""Summarise labelled bench.py JSON lines (A/B and sweep logs): slices/s, ms/step, per-slice loader
and writer CPU time, cgroup CPU usage. Usage: python tools/show_bench_lines.py <log>"""
import json,sys
lab=None
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); c=d['config']; s=c['rank0_stage_s']; n=c['global_batch']*d['steps']
        print('%-16s %7d %6.3f  load_cpu %.1f us/slice  write_cpu %.1f us/pair  slot_cpu %.2f ms/step  proc_cpu %s ms/step  cg %s'%(
            lab, d['value'], d['ms_per_step'], s['load_cpu_s']/n*1e6, s['write_cpu_s']/n*1e6,
            s.get('slot_cpu_s', 0)*1e3/d['steps'], c.get('rank0_process_cpu_ms_per_step'), c.get('cgroup_cpu_ms_per_step')))
    else: lab=l.strip()
