#!/bin/bash
# Round 5: the octree split restricted to device-resident batches -- extraction parity, then the
# full bench line (all legs: host boundary, C2, host-fed, C5, tracking).
set -o pipefail
O=gpurun_out/r5f1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_host_register.py -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo done
