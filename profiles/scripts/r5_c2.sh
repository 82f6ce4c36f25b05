#!/bin/bash
# Round 5: the latency schedule for single images -- parity tests, then the C2 A/B.
set -o pipefail
O=gpurun_out/${R5C2_OUT:-r5c2}
mkdir -p $O
# (parity ran in r5c2 before this A/B)
# timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py -m gpu -k "latency_schedule or batch_equals_single or octree_launch_split" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/scripts/r5_c2_sched.py 3 > $O/c2.txt 2>&1 || exit 1
echo done
