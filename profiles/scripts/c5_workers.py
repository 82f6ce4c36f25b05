"""BASELINE config C5's leg (bench.c5_leg: extraction + SearchLocalPoints per frame, host buffers)
at several caller counts per GPU. python profiles/scripts/c5_workers.py 1 2 4 8"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    torch.cuda.set_device(0)
    for w in [int(v) for v in sys.argv[1:]] or [1, 2, 4, 8]:
        args = SimpleNamespace(nfeatures=2000, c5_workers=w, no_cpu=True)
        r = bench.c5_leg(args, 1, 0, torch.device("cuda", 0))
        print(json.dumps({"workers": w, "frames_per_s": r["frames_per_s"],
                          "one_caller_host_map": r["frames_per_s_one_caller_host_map"], "same": r["resident_map_equals_host_map"],
                          "device_us_per_search": r["device_us_per_search"]}), flush=True)


if __name__ == "__main__":
    main()
