#!/bin/bash
# Round 5: the whole -m gpu suite with the octree launch split on by default; bench A/B of the two
# octree launches' LDS budgets (orbfe_debug_set_octree_lds HI,LO), interleaved; then the host-fed
# experiments (profiles/scripts/r5_hostfed.sh).
set -o pipefail
O=gpurun_out/r5ol
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in 80,40 64,40 64,32; do
    timeout -k 10 200 python bench.py --no-legs --no-cpu --octree-lds $v > $O/lds_${v/,/_}_$i.json 2>&1 || exit 1
  done
done
bash profiles/scripts/r5_hostfed.sh || exit 1
echo done
