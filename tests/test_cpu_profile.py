"""The in-process CPU sampler (src/runtime/cpu_sampler.cpp, bench.py --cpu-profile) and its reader
(tools/cpu_profile.py) on the CPU: the engine's host-only mode runs the real loader / writer pool and
slot threads, the sampler records them, and the reader attributes the samples by thread group, pool
task and loader / writer phase (the table behind profiles/r6/cpu_floor.txt)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_cpu_profile_host_only(tmp_path):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    prof = tmp_path / "prof"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--host-only", "--steps", "100", "--warmup", "2",
           "--no-secondary", "--wipe-passes", "0", "--single-passes", "0", "--cli-runs", "0", "--numa-data", "off",
           "--threads", "4", "--data-root", str(tmp_path / "data"), "--out-root", str(tmp_path / "out"),
           "--cpu-profile", str(prof), "--cpu-profile-period-us", "500"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    dump = tmp_path / "prof.rank0"
    head = dump.read_text().splitlines()
    assert head[0] == "# nm03 cpu samples v2"
    nsamp = int(head[2].split()[1])
    assert nsamp > 50, head[:3]
    assert any(l.startswith("thread ") and l.endswith(" nm03-pool") for l in head)
    assert any(l.startswith("map ") and "libnm03" in l for l in head)
    js = tmp_path / "p.json"
    t = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "cpu_profile.py"), str(dump), "--top", "5",
                        "--json", str(js)], capture_output=True, text=True, timeout=600)
    assert t.returncode == 0, t.stderr[-3000:]
    out = t.stdout
    for section in ("samples by thread group", "nm03-pool by task", "DICOM load by phase",
                    "JPEG pair write by phase"):
        assert section in out, out[:2000]
    # the loader's page-cache read and the writer's file writes are attributed (symbolised frames)
    assert "pread" in out and ("pwritev" in out or "write" in out), out[:3000]
    rec = json.loads(js.read_text())
    assert rec, "empty JSON summary"
