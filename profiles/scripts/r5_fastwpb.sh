#!/bin/bash
# Round 5: k_fast cells per workgroup (side-stream launches, remaining launch) with the octree split
# in place, interleaved; each line checks its last sub-batch against the oracle.
set -o pipefail
O=gpurun_out/r5fw
mkdir -p $O
for i in 1 2; do
  for v in 4,1 2,1 1,1 4,2 8,1; do
    timeout -k 10 200 python bench.py --no-legs --no-cpu --fast-wpb $v > $O/wpb_${v/,/_}_$i.json 2>&1 || exit 1
  done
done
echo done
