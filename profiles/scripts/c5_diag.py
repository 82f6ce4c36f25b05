import sys, time
sys.path.insert(0, '.')
import numpy as np
from orb_slam2_2021_amd import ORBextractor, ORBmatcher, synth_frame
from orb_slam2_2021_amd import synthetic as S
ext = ORBextractor(2000, 1.2, 8, 12, 7)
sc, s2 = ext.GetScaleFactors(), ext.GetScaleSigmaSquares()
k0, d0 = ext(synth_frame(7, 480, 640))
rng = np.random.default_rng(0x50C0DE)
F0 = S.make_frame(k0, d0, sc, s2, 480, 640, S.ARDUCAM_CAM, rng, mp_frac=0.0, tcw=S.pose(tx=0.1, yaw=0.02))
G = S.make_local_map(F0, 50000, rng)
m = ORBmatcher(0.8, True)
for idx, tcw in [(7, S.pose(tx=0.1, yaw=0.02)), (7, S.pose(tx=0.102, yaw=0.021)), (100, S.pose(tx=0.1, yaw=0.02)), (101, S.pose(tx=0.102, yaw=0.021))]:
    k, d = ext(synth_frame(idx, 480, 640))
    F = S.Frame(keys_un=k, descriptors=d, u_right=np.full(len(k), -1.0, np.float32), mp_state=np.zeros(len(k), np.uint8),
                scale_factors=sc, level_sigma2=s2, min_x=0.0, max_x=640.0, min_y=0.0, max_y=480.0, tcw=tcw, **S.ARDUCAM_CAM)
    m.SearchLocalPoints(F, G, 3.0)
    t0 = time.perf_counter()
    nm, best, nv, _ = m.SearchLocalPoints(F, G, 3.0)
    dt = time.perf_counter() - t0
    print(idx, tcw[0, 3], nm, nv, m.last_stats(), round(dt * 1e3, 3), "ms", flush=True)
