import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from orb_slam2_2021_amd import ORBextractor, synth_frame
ext = ORBextractor(2000, 1.2, 8, 20, 7, device=0)
imgs = [synth_frame(i, 376, 1241) for i in range(8)]
ext.extract_batch(np.stack(imgs))
for l in range(8):
    c = [len(ext.debug_candidates(l, i)) for i in range(8)]
    print(l, c)
