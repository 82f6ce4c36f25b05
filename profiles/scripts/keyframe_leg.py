"""Run bench.py's keyframe-search leg alone (SearchByBoW, the relocalisation / Sim3 projections, Fuse,
SearchBySim3, SearchForInitialization, ComputeDistinctiveDescriptors), for rocprofv3 and quick checks."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    print(json.dumps(bench.keyframe_leg(argparse.Namespace(no_cpu=a.no_cpu), reps=a.reps), indent=1))
