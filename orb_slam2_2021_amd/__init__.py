"""orb_slam2_2021_amd -- MI355X-native ORB front-end for ORB-SLAM2 (lreithmayr/ORB_SLAM2_2021).

The product is liborbfe.so (HIP kernels for gfx950 behind the C ABI in include/orbfe.h); this
package is its host-side mirror of the reference's ORBextractor / ORBmatcher interfaces.
"""
from ._lib import (KEYPOINT_DTYPE, LIB_PATH, LibraryMissing, OrbfeError, ORBFE_MP_BAD, ORBFE_MP_NONE,
                   ORBFE_MP_OBSERVED, ORBFE_MP_PRESENT, ORBFE_RESIZE_SCALAR, ORBFE_RESIZE_SIMD128,
                   MPF_BAD, MPF_OBSERVED, MPF_OUTLIER, MPF_PRESENT, MPF_SEEN, MPF_SKIP,
                   MPF_TRACK_IN_VIEW)
from .extractor import ORBextractor, register_host, synth_frame, synth_sequence_frame, unregister_host
from .frames import (FeatureVector, Frame, KeyFrame, KeyFrameMapPoints, LastFrameMapPoints,
                     LocalMapPoints, MapPointGeometry)
from .matcher import ORBmatcher

__all__ = ["ORBextractor", "ORBmatcher", "Frame", "KeyFrame", "FeatureVector", "LocalMapPoints",
           "LastFrameMapPoints", "MapPointGeometry", "KeyFrameMapPoints", "KEYPOINT_DTYPE",
           "synth_frame", "synth_sequence_frame", "register_host", "unregister_host", "OrbfeError", "LibraryMissing"]
