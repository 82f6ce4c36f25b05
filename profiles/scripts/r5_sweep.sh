#!/bin/bash
# Round 5: SearchByProjection's claim order in k_sbp_sweep -- the matcher parity tests, then the C5
# device time per search against the grid-wide rounds (ORBFE_SBP_SWEEP=0), interleaved.
set -o pipefail
O=gpurun_out/r5sweep
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_match.py \
  tests/test_gpu_frustum.py tests/test_gpu_keyframe.py tests/test_gpu_resident_map.py -m gpu > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python profiles/scripts/c5_only.py 4 --resident > $O/c5_sweep_$rep.txt 2>&1 || exit 1
  ORBFE_SBP_SWEEP=0 timeout -k 10 120 python profiles/scripts/c5_only.py 4 --resident > $O/c5_rounds_$rep.txt 2>&1 || exit 1
done
timeout -k 10 120 python profiles/scripts/c5_only.py 2 --resident --per-kernel > $O/c5_kernels.txt 2>&1 || exit 1
echo done
