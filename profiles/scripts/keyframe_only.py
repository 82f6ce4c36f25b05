"""bench.py's keyframe-search leg alone (each ORBmatcher keyframe search per host-buffer call, GPU
vs the oracle): python profiles/scripts/keyframe_only.py [--no-cpu]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    args = bench.parse([a for a in sys.argv[1:]])
    print(json.dumps(bench.keyframe_leg(args)), flush=True)
