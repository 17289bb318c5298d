#!/usr/bin/env python3
"""Engine throughput from Python with or without torch loaded first (which HIP runtime the native
library binds to: torch's bundled libamdhip64 vs /opt/rocm's). Usage: runtime_ab.py DATA_ROOT [torch]"""
import importlib.util
import json
import os
import sys
import time

root = sys.argv[1]
if len(sys.argv) > 2 and sys.argv[2] == "torch":
    import torch  # noqa: F401
here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libdir = os.path.join(here, "nm03_capstone_project_amd", "lib")
so = [f for f in os.listdir(libdir) if f.startswith("_nm03") and f.endswith(".so")][0]
spec = importlib.util.spec_from_file_location("_nm03", os.path.join(libdir, so))
n = importlib.util.module_from_spec(spec)
spec.loader.exec_module(n)
base = n.cohort_dir(root)
items = []
for p in n.find_patient_dirs(base):
    _, files = n.list_patient_series(base, p)
    od = f"/tmp/rab_out/{p}"
    os.makedirs(od, exist_ok=True)
    items += [(f, od) for f in files]
wl = n.WorkList(items)
cfg = n.EngineConfig()
cfg.batch_size, cfg.streams, cfg.threads = 64, 6, 16
eng = n.Engine(cfg)
for _ in range(3):
    eng.run_list(wl)
steps = 20
t = time.perf_counter()
agg = {"load_s": 0.0, "write_s": 0.0, "wall_s": 0.0}
for _ in range(steps):
    _, _, tm = eng.run_list(wl)
    for k in agg:
        agg[k] += tm[k]
dt = time.perf_counter() - t
print(json.dumps({"torch_first": "torch" in sys.modules, "ms_per_step": round(dt / steps * 1e3, 3),
                  "slices_per_s": round(len(items) * steps / dt), **{k: round(v / steps * 1e3, 3) for k, v in agg.items()}}))
