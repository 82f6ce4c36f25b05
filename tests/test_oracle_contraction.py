"""The reference is built with -O3 -march=native (CMakeLists.txt), where GCC's default
-ffp-contract=fast may fuse float multiply-adds; the oracle checker (and the GPU path) round every
operation separately. The same oracle source built with the reference's flags (liborbref_native.so)
shows what contraction changes on this path: nothing in keypoints or descriptors on KITTI-shaped
frames, and keypoint angles (fastAtan2's polynomial) within one float ulp -- up to 3.05e-5 degree
near 360, above the 1e-5 the north star allows, so the angle bar holds against the restatement, not
against an FMA-contracted build."""
import numpy as np

from orb_slam2_2021_amd import synth_frame
from oracle.orbref import RefExtractor


def test_fma_contracted_build_differs_only_in_angle_ulps():
    for i in (0, 3):
        img = synth_frame(i, 376, 1241)
        ka, da = RefExtractor(2000, 1.2, 8, 20, 7)(img)
        kb, db = RefExtractor(2000, 1.2, 8, 20, 7, kind="native")(img)
        assert len(ka) == len(kb) > 2000
        for f in ("x", "y", "size", "response", "octave", "class_id"):
            assert np.array_equal(ka[f], kb[f]), f
        assert np.array_equal(da, db)
        ulp = np.spacing(np.maximum(np.abs(ka["angle"]), np.float32(1)).astype(np.float32))
        assert np.all(np.abs(ka["angle"] - kb["angle"]) <= ulp)
