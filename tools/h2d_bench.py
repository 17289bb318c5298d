#!/usr/bin/env python3
"""Host→device copy throughput on the box: pinned 8.4 MB copies (one engine batch of 64 slices),
serial on one stream and concurrent on 6 streams. Run once per copy-engine setting, e.g.
  python tools/h2d_bench.py; HSA_ENABLE_SDMA=0 python tools/h2d_bench.py
Prints one JSON line."""
import json
import os
import time

import torch


def main():
    n = 64 * 256 * 256 * 2 + 64 * 1024
    reps = 48
    dev = torch.device("cuda:0")
    host = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(6)]
    devb = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(6)]
    streams = [torch.cuda.Stream() for _ in range(6)]
    res = {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default"), "bytes": n}
    for s in range(6):  # warm
        with torch.cuda.stream(streams[s]):
            devb[s].copy_(host[s], non_blocking=True)
    torch.cuda.synchronize()
    for label, ns in (("serial_1stream", 1), ("concurrent_6streams", 6)):
        t0 = time.perf_counter()
        for r in range(reps):
            s = r % ns
            with torch.cuda.stream(streams[s]):
                devb[s].copy_(host[s], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[label + "_GBps"] = round(n * reps / dt / 1e9, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
