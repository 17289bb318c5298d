#!/usr/bin/env python3
"""Wall clock of repeated unmodified CLI invocations (hyperfine-style, README.md:92-96 of the
reference): python tools/cli_wall.py BIN_DIR DATA_ROOT [RUNS] [CLI ...]. One JSON line per CLI.

Each run is reaped with os.wait4 (nm03_capstone_project_amd/utils/cli_wall.py): exact wall time
and the child's rusage, no 50 ms polling quantum."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nm03_capstone_project_amd.utils.cli_wall import time_cli  # noqa: E402

b, root = sys.argv[1], sys.argv[2]
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 10
clis = sys.argv[4:] or ["img_processing_parallel", "img_processing_sequential", "test_pipeline"]
for exe in clis:
    js = f"/tmp/bl_cli_{exe}.json"
    res = time_cli([f"{b}/{exe}", "--data-root", root, "--out", f"/tmp/bl_cli_{exe}", "--quiet", "--json", js],
                   runs=runs, json_path=js)
    print(json.dumps({"cli": exe, **res}), flush=True)
