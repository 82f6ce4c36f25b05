"""bench.py's tracking leg alone (Tracking's per-frame device sequence): python
profiles/scripts/tracking_only.py [--no-cpu]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    args = bench.parse([a for a in sys.argv[1:]])
    print(json.dumps(bench.tracking_leg(args)), flush=True)
