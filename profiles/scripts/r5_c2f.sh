#!/bin/bash
# Round 5: where the latency schedule's side work is enqueued (after 0 / 1 / 2 more resize launches):
# parity, then the C2 A/B.
set -o pipefail
O=gpurun_out/r5c2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py -m gpu -k "latency_schedule or small_device_batch" > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u profiles/scripts/r5_c2_sched.py 3 > $O/c2.txt 2>&1 || exit 1
echo done
