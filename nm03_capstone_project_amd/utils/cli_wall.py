"""Exact wall clock of whole CLI invocations, the way the reference measured its binaries
(hyperfine / `time`, /root/reference/README.md:92-96).

`subprocess.run(..., timeout=...)` waits in `Popen.wait(timeout)`, which polls with sleeps of up
to 50 ms: every figure it produced was quantised to 50 ms steps. Here the
child is reaped with one blocking `os.wait4`, so the wall clock ends when the child does, and the
child's own rusage (user/sys CPU, max RSS) comes with it. A hang is bounded by a watchdog thread
that kills the child, not by polling.
"""
import json
import os
import subprocess
import tempfile
import threading
import time


def run_once(argv, timeout_s=120.0, env=None):
    """Run argv once; returns {rc, wall_s, user_s, sys_s, maxrss_kb, stderr_tail}."""
    with tempfile.TemporaryFile() as err:
        launch_unix = time.time()
        t0 = time.perf_counter()
        p = subprocess.Popen(argv, stdout=subprocess.DEVNULL, stderr=err, env=env)
        done = threading.Event()

        def watchdog():
            if not done.wait(timeout_s):
                try:
                    p.kill()
                except OSError:
                    pass

        w = threading.Thread(target=watchdog, daemon=True)
        w.start()
        _, status, ru = os.wait4(p.pid, 0)
        wall = time.perf_counter() - t0
        done.set()
        p.returncode = os.waitstatus_to_exitcode(status)  # reaped here: Popen must not wait again
        err.seek(0)
        tail = err.read()[-400:].decode(errors="replace")
    return {"rc": p.returncode, "wall_s": round(wall, 6), "user_s": round(ru.ru_utime, 6),
            "sys_s": round(ru.ru_stime, 6), "maxrss_kb": ru.ru_maxrss, "stderr_tail": tail,
            "launch_unix_s": launch_unix}


def time_cli(argv, runs=10, json_path=None, timeout_s=120.0, env=None):
    """`runs` invocations of argv. If json_path is given, argv must write the CLI's --json record
    there; its phase split (hip_init_s, engine_ctor_s, processing_wall_s, ...) is collected too.
    Returns a summary: median/min/max wall, per-run rows, and the median of each phase."""
    rows = []
    for _ in range(runs):
        if json_path and os.path.exists(json_path):
            os.unlink(json_path)
        r = run_once(argv, timeout_s, env)
        if json_path and os.path.exists(json_path):
            try:
                with open(json_path) as f:
                    r["phases"] = json.load(f)
            except (OSError, ValueError):
                pass
            ph = r.get("phases") or {}
            main_unix = ph.pop("main_unix_s", None)
            if isinstance(main_unix, (int, float)):
                # exec → main: dynamic loading of the CLI and its libraries, before any of our code
                ph["pre_main_s"] = round(main_unix - r["launch_unix_s"], 6)
        rows.append(r)
    walls = sorted(r["wall_s"] for r in rows)
    ok = all(r["rc"] == 0 for r in rows)
    out = {"runs": runs, "all_ok": ok, "wall_median_s": walls[len(walls) // 2], "wall_min_s": walls[0],
           "wall_max_s": walls[-1], "walls_s": [r["wall_s"] for r in rows],
           "cpu_median_s": sorted(r["user_s"] + r["sys_s"] for r in rows)[len(rows) // 2]}
    phases = {}
    for r in rows:
        for k, v in (r.get("phases") or {}).items():
            if k.endswith("_s") and isinstance(v, (int, float)):
                phases.setdefault(k, []).append(v)
    if phases:
        out["phases_median_s"] = {k: round(sorted(v)[len(v) // 2], 6) for k, v in sorted(phases.items())}
    if not ok:
        out["failures"] = [{"rc": r["rc"], "stderr_tail": r["stderr_tail"]} for r in rows if r["rc"] != 0][:2]
    return out
