"""CLIs on CPU: test_pipeline --cpu (BASELINE config 1, golden plumbing) and argument handling."""
import io
import os
import re

import numpy as np
import pytest

from conftest import run_bin


def test_test_pipeline_cpu(native, cohort_root, tmp_path):
    out = tmp_path / "out-test"
    (out).mkdir()
    (out / "stale.jpg").write_bytes(b"x")
    r = run_bin("test_pipeline", "--cpu", "--data-root", cohort_root, "--out", str(out))
    assert r.returncode == 0, r.stderr
    names = sorted(p.name for p in out.iterdir())
    assert names == sorted(["original_image.jpg", "preprocessed_image.jpg", "segmentation.jpg", "erosion_result.jpg",
                            "final_dilated_result.jpg", "multi_view.jpg"])
    # golden_run gives the same original/dilated exports
    raw, meta = native.read_slice(native.test_slice_path(cohort_root))
    g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                          native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
    assert (out / "original_image.jpg").read_bytes() == g["jpeg_original"]
    assert (out / "final_dilated_result.jpg").read_bytes() == g["jpeg_processed"]
    PIL = pytest.importorskip("PIL.Image")
    im = PIL.open(io.BytesIO((out / "multi_view.jpg").read_bytes()))
    assert im.size == (2560, 512)


@pytest.mark.parametrize("flag,mode,layer", [("gray", "L", None), ("444", "RGB", (1, 1, 1, 0)),
                                              ("420", "RGB", (1, 2, 2, 0))])
def test_test_pipeline_cpu_jpeg_sampling(native, cohort_root, tmp_path, flag, mode, layer):
    """--jpeg-sampling: every export (and the montage) in the chosen layout, equal to golden_run
    with RenderParams.jpeg_sampling set."""
    out = tmp_path / "o"
    r = run_bin("test_pipeline", "--cpu", "--jpeg-sampling", flag, "--data-root", cohort_root, "--out", str(out))
    assert r.returncode == 0, r.stderr
    rp = native.RenderParams()
    rp.jpeg_sampling = {"420": 0, "444": 1, "gray": 2}[flag]
    raw, meta = native.read_slice(native.test_slice_path(cohort_root))
    g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                          native.PipelineParams(), rp, meta["spacing_x"], meta["spacing_y"])
    assert (out / "original_image.jpg").read_bytes() == g["jpeg_original"]
    assert (out / "final_dilated_result.jpg").read_bytes() == g["jpeg_processed"]
    PIL = pytest.importorskip("PIL.Image")
    for name in ("original_image.jpg", "segmentation.jpg", "multi_view.jpg"):
        im = PIL.open(io.BytesIO((out / name).read_bytes()))
        assert im.mode == mode
        if layer:
            assert im.layer[0] == layer
    r = run_bin("test_pipeline", "--cpu", "--jpeg-sampling", "422", "--data-root", cohort_root, "--out", str(out))
    assert r.returncode == 2 and "--jpeg-sampling" in r.stderr


def test_test_pipeline_html_viewer(cohort_root, tmp_path):
    """--html: the reference's 5-view window (MultiViewWindow 2300x450) as a page over the exported
    stage images."""
    out = tmp_path / "o"
    r = run_bin("test_pipeline", "--cpu", "--html", "--data-root", cohort_root, "--out", str(out))
    assert r.returncode == 0, r.stderr
    page = (out / "multi_view.html").read_text()
    assert "width:2300px;height:450px" in page
    for name in ("original_image", "preprocessed_image", "segmentation", "erosion_result", "final_dilated_result"):
        assert f'src="{name}.jpg"' in page and (out / f"{name}.jpg").exists()


def test_cli_help_and_bad_flag():
    for tool in ("test_pipeline", "img_processing_sequential", "img_processing_parallel"):
        r = run_bin(tool, "--help")
        assert r.returncode == 0 and "--data-root" in r.stdout
        r = run_bin(tool, "--bogus")
        assert r.returncode == 2


def test_synth_tool(tmp_path):
    r = run_bin("nm03_synth", "--data-root", str(tmp_path), "--patients", "2", "--min-slices", "2", "--max-slices", "3")
    assert r.returncode == 0, r.stderr
    assert "Wrote" in r.stdout


def test_missing_data_root_is_fatal(tmp_path):
    r = run_bin("test_pipeline", "--cpu", "--data-root", str(tmp_path / "nope"), "--out", str(tmp_path / "o"))
    assert r.returncode == 1 and "Fatal error" in r.stderr


def test_numa_cpulist_parsing(native):
    """Host NUMA placement (numa.h): sysfs cpulists such as node0 of an MI355X node."""
    assert native.numa_parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert native.numa_parse_cpulist("0-63,128-191")[-1] == 191
    assert native.numa_parse_cpulist("") == []
    assert native.numa_node_cpus(-1) == []


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int16, np.float32])
def test_metaimage_roundtrip(native, tmp_path, dtype):
    a = (np.arange(3 * 5 * 7) % 200).astype(dtype).reshape(3, 5, 7)
    native.mhd_write(str(tmp_path / "vol"), a, 0.5, 0.75, 2.0)
    b, sp = native.mhd_read(str(tmp_path / "vol.mhd"))
    assert b.dtype == a.dtype and np.array_equal(a, b) and sp == (0.5, 0.75, 2.0)
    native.mhd_write(str(tmp_path / "img"), a[1].copy())
    c, _ = native.mhd_read(str(tmp_path / "img.mhd"))
    assert np.array_equal(c, a[1])
    assert "NDims = 2" in (tmp_path / "img.mhd").read_text()


def test_test_pipeline_dump_mhd_cpu(native, cohort_root, tmp_path):
    """--dump-mhd writes the stage arrays; they equal the golden model of the same slice."""
    dump = tmp_path / "mhd"
    r = run_bin("test_pipeline", "--cpu", "--data-root", cohort_root, "--out", str(tmp_path / "o"),
                "--dump-mhd", str(dump))
    assert r.returncode == 0, r.stderr
    raw, meta = native.read_slice(native.test_slice_path(cohort_root))
    g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"])
    inp, _ = native.mhd_read(str(dump / "input.mhd"))
    assert np.array_equal(inp.view(np.uint16), raw)
    sh, _ = native.mhd_read(str(dump / "sharpened.mhd"))
    assert np.array_equal(sh, g["sharpened"])
    for name, key in (("band", "band"), ("segmentation", "region"), ("dilation", "dilated")):
        m, _ = native.mhd_read(str(dump / f"{name}.mhd"))
        assert np.array_equal(m.astype(bool), np.asarray(g[key]).astype(bool)), name


def test_volume_cli_cpu_golden(native, cohort_root, tmp_path):
    """--mode 3d --cpu: the golden 3D oracle of the GPU 3D export (BASELINE config 5): one volume
    per patient, 3D SRG + 7×7×7 dilation by default, two JPEGs per plane, JSON per patient."""
    import json
    out, js = tmp_path / "o", tmp_path / "v.json"
    r = run_bin("img_processing_parallel", "--mode", "3d", "--cpu", "--data-root", cohort_root, "--out", str(out),
                "--json", str(js))
    assert r.returncode == 0, r.stderr
    assert "=== Starting 3D Volume Processing for All Patients ===" in r.stdout
    assert "Successfully processed 4/4 patients." in r.stdout
    j = json.load(open(js))
    assert j["dilation_size"] == 7 and j["connectivity"] == 6 and j["backend"] == "cpu"
    base = native.cohort_dir(cohort_root)
    n = sum(len(native.list_patient_series(base, p)[1]) for p in native.find_patient_dirs(base))
    assert j["slices"] == n and len(list(out.rglob("*.jpg"))) == 2 * n
    PIL = pytest.importorskip("PIL.Image")
    for f in list(out.rglob("*_processed.jpg"))[:3]:
        assert PIL.open(io.BytesIO(f.read_bytes())).size == (512, 512)
    r = run_bin("img_processing_parallel", "--mode", "3d", "--cpu", "--dilation-size", "3", "--data-root", cohort_root,
                "--out", str(tmp_path / "o3"), "--json", str(js))
    assert r.returncode == 0 and json.load(open(js))["dilation_size"] == 3


def _tree(root):
    return {str(p.relative_to(root)): p.read_bytes() for p in sorted(root.rglob("*.jpg"))}


@pytest.mark.parametrize("ranks,conn", [(2, "6"), (3, "26"), (4, "6")])
def test_volume_cli_cpu_split_volume_identical(native, cohort_root, tmp_path, ranks, conn):
    """--mode 3d --cpu --split-volume --gpus N: every volume cut into z-slabs over N rank processes
    (host comm), boundary planes and dilation halos exchanged (volume_slabs.h) — byte-identical to
    the single-process golden 3D output (thin slabs included: 3–5 planes, dilation radius 3)."""
    import json
    ref, out = tmp_path / "ref", tmp_path / "split"
    r = run_bin("img_processing_parallel", "--mode", "3d", "--cpu", "--srg-connectivity", conn, "--data-root",
                cohort_root, "--out", str(ref), "--quiet")
    assert r.returncode == 0, r.stderr
    r = run_bin("img_processing_parallel", "--mode", "3d", "--cpu", "--split-volume", "--gpus", str(ranks),
                "--srg-connectivity", conn, "--data-root", cohort_root, "--out", str(out), "--quiet", "--json",
                str(tmp_path / "s.json"))
    if ranks > 3:  # the cohort has 3–5 planes per patient: a too-thin volume fails, the rest succeed
        assert r.returncode == 0, r.stderr
        j = json.load(open(tmp_path / "s.json"))
        bad = [p for p in j["patients"] if not p["ok"]]
        assert bad and all(p["slices"] == 0 for p in bad)
        assert "cannot be split over 4 ranks" in r.stderr
        return
    assert r.returncode == 0, r.stderr
    t = _tree(ref)
    assert len(t) > 0 and _tree(out) == t
    j = json.load(open(tmp_path / "s.json"))
    assert j["split_volume"] and j["gpus"] == ranks and all(p["ok"] for p in j["patients"])


@pytest.mark.parametrize("cli,args", [
    ("test_pipeline", ["--cpu"]),
    ("img_processing_parallel", ["--mode", "3d", "--cpu"]),
    ("test_pipeline", ["--cpu", "--input", "/nonexistent/slice.dcm"]),
])
def test_fast_exit_same_output(native, cohort_root, tmp_path, cli, args):
    """The CLIs end with cli_exit (flush, then _exit without teardown): stdout, stderr, exit code and
    the output tree are the same as with the normal return (NM03_FAST_EXIT=0), also on failure."""
    res = []
    for fx in ("1", "0"):
        out = tmp_path / f"o{fx}"
        r = run_bin(cli, *args, "--data-root", cohort_root, "--out", str(out), env={"NM03_FAST_EXIT": fx})
        tree = {}
        if out.exists():
            for p in sorted(out.rglob("*")):
                if p.is_file():
                    tree[str(p.relative_to(out))] = p.read_bytes()
        norm = lambda t: re.sub(r"\d+(\.\d+)? (ms|s)\b", "T", t.replace(str(out), "OUT"))  # timings
        res.append((r.returncode, norm(r.stdout), norm(r.stderr), tree))
    assert res[0] == res[1]
    assert res[0][1] or res[0][2]  # something was printed and survived the fast exit


def test_native_bench_cohort_host_only(native, cohort_root, tmp_path):
    """nm03_bench --config cohort --host-only (the sanitizer sweep's engine run): every slice loaded
    and both JPEGs written per slice, no GPU."""
    import json
    out = tmp_path / "o"
    r = run_bin("nm03_bench", "--config", "cohort", "--host-only", "--data-root", cohort_root, "--out", str(out),
                "--steps", "2", "--warmup", "1", "--threads", "4", "--streams", "2", "--batch-size", "8")
    assert r.returncode == 0, r.stderr
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["slices_per_s"] > 0 and rec["kernels_s"] == 0
    n = rec["slices_per_step"]
    files = [p for d in out.iterdir() for p in d.iterdir()]
    assert len(files) == 2 * n and all(p.read_bytes()[:2] == b"\xff\xd8" for p in files)


def test_parallel_default_rank_count_policy(native, cohort_root):
    """img_processing_parallel without --gpus (auto): one rank per kAutoSlicesPerRank slices of the
    cohort, at least 1, at most every visible GPU; the count comes from directory listings only."""
    per = native.auto_slices_per_rank()
    assert per == 4096
    assert native.auto_gpus(465, 8) == 1          # the T1+C cohort: one GPU
    assert native.auto_gpus(per, 8) == 1 and native.auto_gpus(per + 1, 8) == 2
    assert native.auto_gpus(10000, 8) == 3        # BASELINE config 4
    assert native.auto_gpus(10 ** 6, 8) == 8      # capped at the visible GPUs
    assert native.auto_gpus(0, 8) == 1 and native.auto_gpus(50000, 0) == 1
    n = native.count_cohort_slices(cohort_root)
    base = native.cohort_dir(cohort_root)
    assert n == sum(len(native.list_patient_series(base, p)[1]) for p in native.find_patient_dirs(base))
    assert native.count_cohort_slices("/nonexistent/") == -1
