"""k_pyramid phase clocks: one 1241x376 image through the extractor 5 times per tiling with a
library built with -DORBFE_PYR_CLOCKS (make -C orb_slam2_2021_amd/csrc OUT=../lib_prof OBJ=../build_prof
EXTRA=-DORBFE_PYR_CLOCKS) and ORBFE_PYR_CLOCKS=1: the middle workgroup prints s_memrealtime deltas
(10 ns units) of its phases -- level fields, table staging, then levels 1..L-1.
usage: ORBFE_LIB=orb_slam2_2021_amd/lib_prof/liborbfe.so ORBFE_PYR_CLOCKS=1 python profiles/scripts/pyr_clocks.py"""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from orb_slam2_2021_amd import ORBextractor, synth_frame
img = synth_frame(3, 376, 1241)
for t in [(16, 12), (32, 24)]:
    e = ORBextractor(2000, 1.2, 8, 20, 7)
    e.debug_set_pyramid_tiles(t, (0, 0))
    for i in range(5):
        e(img)
    print("tiles", t, flush=True)
