"""Run the C5-shape SearchLocalPoints leg (isInFrustum + SearchByProjection) alone, for rocprofv3."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

if __name__ == "__main__":
    a = argparse.Namespace(nfeatures=2000, no_cpu=True)
    print(bench.sbp_leg(a, reps=5))
