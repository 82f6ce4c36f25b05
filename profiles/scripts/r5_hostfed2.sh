#!/bin/bash
# Round 5: host-fed C3 leg, one vs two copy streams per sub-batch (16 input slots), interleaved.
set -o pipefail
O=gpurun_out/r5hf2
mkdir -p $O
HF="--feed host --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu --event-every 1000000 --input-slots 16"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c3.py -k host_fed -m gpu > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py $HF --copy-streams 1 > $O/cs1_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py $HF --copy-streams 2 > $O/cs2_$i.json 2>&1 || exit 1
done
echo done
