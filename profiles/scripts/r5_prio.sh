#!/bin/bash
# Round 5: which pipeline streams run at high priority (the resize chain on the extraction streams
# vs FAST on the shared side stream), interleaved.
set -o pipefail
O=gpurun_out/r5pr
mkdir -p $O
for i in 1 2; do
  for v in side,match extract,match extract,side,match extract; do
    timeout -k 10 200 python bench.py --no-legs --no-cpu --high-prio $v > $O/p_${v//,/_}_$i.json 2>&1 || exit 1
  done
done
echo done
