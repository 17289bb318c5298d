"""utils/cli_wall: exact wall clock (wait4, no 50 ms polling quantum), exit codes, phase split."""
import json
import sys

from nm03_capstone_project_amd.utils.cli_wall import run_once, time_cli


def test_wall_is_not_quantised():
    # A 7 ms child must read as ≈7 ms, not 50 ms (Popen.wait(timeout) polling would give 0.05+).
    r = run_once(["sleep", "0.007"])
    assert r["rc"] == 0
    assert 0.007 <= r["wall_s"] < 0.045, r
    assert r["user_s"] >= 0 and r["maxrss_kb"] > 0


def test_exit_code_and_stderr():
    r = run_once([sys.executable, "-c", "import sys; sys.stderr.write('boom'); sys.exit(3)"])
    assert r["rc"] == 3 and "boom" in r["stderr_tail"]


def test_watchdog_kills_a_hang():
    r = run_once([sys.executable, "-c", "import time; time.sleep(30)"], timeout_s=0.3)
    assert r["rc"] < 0 and r["wall_s"] < 5


def test_phase_split_collected(tmp_path):
    js = tmp_path / "cli.json"
    code = ("import json,sys; json.dump({'hip_init_s': 0.1, 'processing_wall_s': 0.02, 'slices': 5}, "
            f"open({str(js)!r}, 'w'))")
    res = time_cli([sys.executable, "-c", code], runs=3, json_path=str(js))
    assert res["all_ok"] and res["runs"] == 3 and len(res["walls_s"]) == 3
    assert res["wall_min_s"] <= res["wall_median_s"] <= res["wall_max_s"]
    assert res["phases_median_s"] == {"hip_init_s": 0.1, "processing_wall_s": 0.02}
    json.dumps(res)
