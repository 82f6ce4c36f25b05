"""Which streams push a handle's two streams onto one hardware queue? One KITTI image through
orbfe_extract on a fresh handle (p50 of 300 calls) after creating K idle torch streams of normal or
of high priority (the runtime's queue pool: the default without ORBFE_DEDICATED_QUEUES).
usage: python profiles/scripts/c2_queues2.py normal|high K ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "profiles", "scripts"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from c2_queues import p50  # noqa: E402
from orb_slam2_2021_amd import ORBextractor, synth_frame  # noqa: E402


def main():
    kind = sys.argv[1]
    ks = [int(a) for a in sys.argv[2:]]
    img = np.ascontiguousarray(synth_frame(3, 376, 1241))
    keep, have = [], 0
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    for k in ks:
        while have < k:
            s = torch.cuda.Stream(priority=hi if kind == "high" else 0)
            with torch.cuda.stream(s):
                torch.zeros(1, device="cuda").add_(1)
            keep.append(s)
            have += 1
        print(f"{kind} idle streams {k}: p50 {p50(ORBextractor(2000, 1.2, 8, 20, 7), img):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
