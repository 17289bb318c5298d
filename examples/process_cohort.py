"""Process a T1+C cohort from Python, like img_processing_parallel on one GPU.

    python examples/process_cohort.py --data-root data/ --out out-py/ [--synth] [--host-only]
                                      [--se-shape disc] [--render-filter nearest] [--jpeg-sampling gray]

--synth writes the synthetic 20-patient cohort first; --host-only runs the host path alone (loads and
JPEG writes with fixed segments, no GPU), which is what the CPU test of this example exercises.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nm03_capstone_project_amd as nm  # noqa: E402
from nm03_capstone_project_amd.utils.cohort import Cohort, synth_cohort  # noqa: E402

SAMPLING = {"420": 0, "444": 1, "gray": 2}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--data-root", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--synth", action="store_true", help="write the synthetic cohort under --data-root first")
    ap.add_argument("--host-only", action="store_true", help="no GPU: host loads and writes only")
    ap.add_argument("--se-shape", choices=("square", "disc"), default="square")
    ap.add_argument("--render-filter", choices=("bilinear", "nearest"), default="bilinear")
    ap.add_argument("--jpeg-sampling", choices=tuple(SAMPLING), default="420")
    a = ap.parse_args(argv)
    if a.synth:
        synth_cohort(a.data_root, patients=4, min_slices=5, max_slices=7)
    cohort = Cohort.discover(a.data_root)
    items = cohort.work_items(a.out)
    cfg = nm.PipelineConfig(se_shape=int(a.se_shape == "disc"), render_filter=int(a.render_filter == "nearest"),
                            jpeg_sampling=SAMPLING[a.jpeg_sampling], host_only=a.host_only)
    pipe = nm.SlicePipeline(cfg)
    t0 = time.perf_counter()
    statuses, _ = pipe.process(items)
    dt = time.perf_counter() - t0
    ok = sum(1 for code, _ in statuses if code == 0)
    for pid, why in cohort.skipped:
        print(f"skipped {pid}: {why}")
    print(f"{len(cohort)} patients, {ok}/{len(items)} slices in {dt * 1e3:.1f} ms -> {a.out}")
    return 0 if ok == len(items) else 1


if __name__ == "__main__":
    sys.exit(main())
