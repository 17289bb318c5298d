#!/usr/bin/env python3
"""Wall clock of repeated unmodified CLI invocations (hyperfine-style, README.md:92-96 of the
reference): python tools/cli_wall.py BIN_DIR DATA_ROOT [RUNS]. One JSON line per run."""
import json
import subprocess
import sys
import time

b, root = sys.argv[1], sys.argv[2]
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 6
for exe in ("img_processing_parallel", "img_processing_sequential", "test_pipeline"):
    for i in range(runs):
        t = time.perf_counter()
        r = subprocess.run([f"{b}/{exe}", "--data-root", root, "--out", f"/tmp/bl_cli_{exe}", "--quiet"],
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=120)
        print(json.dumps({"cli": exe, "run": i, "rc": r.returncode, "wall_s": round(time.perf_counter() - t, 4)}),
              flush=True)
