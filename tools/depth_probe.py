"""Host-only engine: run latency and stage times per queued run at a given pipeline depth (diagnosis of deep pipelining)."""
import os, sys, time
sys.path.insert(0, '/root/repo')
import nm03_capstone_project_amd as nm
n = nm.native()
root = os.environ.get('DP_ROOT', '/dev/shm/dp_data/')
if not os.path.exists(root):
    n.synth_cohort(root, threads=16)
base = n.cohort_dir(root)
def items_for(out):
    its = []
    for pid in n.find_patient_dirs(base):
        _, files = n.list_patient_series(base, pid)
        d = os.path.join(out, pid); os.makedirs(d, exist_ok=True)
        its += [(f, d) for f in files]
    return its
depth = int(sys.argv[1]); steps = int(sys.argv[2])
cfg = nm.PipelineConfig(batch_size=96, streams=4, threads=int(os.environ.get('DP_THREADS', '16'))).engine_config(); cfg.host_only = True
eng = n.Engine(cfg)
works = [n.WorkList(items_for(os.environ.get('DP_OUT', '/dev/shm/dp_out') + f'/t{k}')) for k in range(depth)]
pending = []; t0 = time.perf_counter(); times = []
for k in range(steps):
    ts = time.perf_counter()
    pending.append((eng.submit(works[k % depth]), ts))
    if len(pending) == depth:
        t, ts0 = pending.pop(0); codes, msgs, st = eng.wait(t); times.append((round((time.perf_counter() - ts0) * 1e3, 1), round(st["load_s"]*1e3,1), round(st["write_s"]*1e3,1), round(st["load_cpu_s"]*1e3,1), round(st["write_cpu_s"]*1e3,1)))
for t, ts0 in pending:
    eng.wait(t)
dt = time.perf_counter() - t0
print(f"depth {depth}: {steps*465/dt:.0f} slices/s; run latencies ms: {times[:12]}")
