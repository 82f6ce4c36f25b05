#!/bin/bash
# Round 5: small host calls after larger ones on one handle (the one-copy / three-copy D2H paths).
set -o pipefail
O=gpurun_out/r5sc
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_extract.py -m gpu -k "small_calls_after_large or latency_schedule or small_device_batch" > $O/tests.log 2>&1 || exit 1
echo done
