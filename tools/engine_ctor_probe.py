import time, sys
sys.path.insert(0, '.')
import torch
import nm03_capstone_project_amd as nm
from nm03_capstone_project_amd._native import native
n = native()
torch.cuda.init(); torch.zeros(1, device='cuda')
for streams in (1, 2, 6, 6, 1):
    for md in (256,):
        pc = nm.PipelineConfig(batch_size=64, streams=streams, threads=16)
        ec = pc.engine_config()
        ec.max_dim = md
        t0 = time.perf_counter(); e = n.Engine(ec); t1 = time.perf_counter(); del e; t2 = time.perf_counter()
        print(f"streams {streams} max_dim {md}: ctor {1e3*(t1-t0):.1f} ms, dtor {1e3*(t2-t1):.1f} ms", flush=True)
