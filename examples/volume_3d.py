"""One DICOM series as a 3D volume on the MI355X: per-slice preprocessing, 6-connected 3D region
growing and a 7×7×7 dilation (BASELINE config 5), checked against the golden 3D model.

    python examples/volume_3d.py --series path/to/series_dir [--ball]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import nm03_capstone_project_amd as nm  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--series", required=True)
    ap.add_argument("--ball", action="store_true", help="digital ball instead of the 7x7x7 cube")
    a = ap.parse_args(argv)
    vp = nm.VolumePipeline(nm.PipelineConfig(se_shape=int(a.ball)), connectivity=6, dilation=7)
    res = vp.run_series(a.series)
    band = res["band"]
    region, dil = vp.golden(band, vp.default_seeds(band))
    same = np.array_equal(res["region"], region) and np.array_equal(res["dilated"], dil)
    print(f"volume {tuple(band.shape)}: region {int(res['region'].sum())} voxels, dilated "
          f"{int(res['dilated'].sum())} voxels, GPU == golden: {same}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
