#!/usr/bin/env python3
"""Interleaved cold-CLI A/B (hyperfine-style walls, one run of each variant per round):

    python tools/cold_ab.py DATA_ROOT ROUNDS NAME=BIN_DIR[:LD_LIBRARY_PATH][@ARG,ARG...] ...

Prints one JSON line per variant: wall median/min and the median of every phase of the CLI's
--json record (hip_init_s, streams_s, engine_ctor_s, plan_s, ...)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nm03_capstone_project_amd.utils.cli_wall import time_cli  # noqa: E402

root, rounds = sys.argv[1], int(sys.argv[2])
variants = []
for v in sys.argv[3:]:
    name, spec = v.split("=", 1)
    spec, _, extra = spec.partition("@")
    bdir, _, lib = spec.partition(":")
    variants.append((name, bdir, lib, [a for a in extra.split(",") if a]))
rows = {n: [] for n, _, _, _ in variants}
for r in range(rounds):
    for name, bdir, lib, extra in variants:
        env = dict(os.environ)
        if lib:
            env["LD_LIBRARY_PATH"] = lib
        js = f"/tmp/cold_ab_{name}.json"
        # outputs on tmpfs like the bench's config.cli_wall (the root overlay serialises small-file writes)
        res = time_cli([f"{bdir}/img_processing_parallel", "--data-root", root, "--out", f"/dev/shm/cold_ab_{name}",
                        "--quiet", "--json", js] + extra, runs=1, json_path=js, env=env)
        rows[name].append(res)
for name, rs in rows.items():
    walls = [x["wall_median_s"] for x in rs]
    ph = {}
    for x in rs:
        for k, v in x.get("phases_median_s", {}).items():
            ph.setdefault(k, []).append(v)
    # per-run differences (medians of separate fields come from different runs)
    diffs = []
    for x in rs:
        p = x.get("phases_median_s", {})
        if "engine_setup_s" in p and "hip_init_s" in p:
            diffs.append(p["engine_setup_s"] - p["hip_init_s"])
    print(json.dumps({"variant": name, "runs": len(rs), "all_ok": all(x["all_ok"] for x in rs),
                      "setup_minus_hip_init_median_s": round(statistics.median(diffs), 6) if diffs else None,
                      "wall_median_s": round(statistics.median(walls), 6), "wall_min_s": round(min(walls), 6),
                      "walls_s": [round(w, 4) for w in walls],
                      "phases_median_s": {k: round(statistics.median(v), 6) for k, v in sorted(ph.items())},
                      "failures": [f for x in rs for f in x.get("failures", [])][:2]}), flush=True)
