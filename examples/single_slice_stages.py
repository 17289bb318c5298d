"""Every stage image of one slice on the MI355X (test_pipeline's view from Python), checked against the
golden CPU model: the GPU result is bit-identical by contract.

    python examples/single_slice_stages.py --dicom path/to/1-14.dcm --out stages/
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import nm03_capstone_project_amd as nm  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--dicom", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    n = nm.native()
    raw, meta = n.read_slice(a.dicom, 0)
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2))
    gpu, ref = pipe.run_array(raw, meta), pipe.golden(raw, meta)
    same = all(np.array_equal(gpu[k], ref[k]) for k in ("band", "region", "eroded", "dilated"))
    os.makedirs(a.out, exist_ok=True)
    names = ("original_image", "preprocessed_image", "segmentation", "erosion_result", "final_dilated_result")
    for name, jpeg in zip(names, gpu["jpegs"]):
        with open(os.path.join(a.out, name + ".jpg"), "wb") as f:
            f.write(jpeg)
    print(f"{raw.shape[1]}x{raw.shape[0]} slice: region {int(gpu['region'].sum())} px, "
          f"dilated {int(gpu['dilated'].sum())} px, GPU == golden: {same}; 5 stage JPEGs in {a.out}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
