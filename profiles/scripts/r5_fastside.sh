#!/bin/bash
# Round 5: FAST levels on the side stream (--fast-side K) x cells per workgroup, interleaved.
set -o pipefail
O=gpurun_out/r5fs
mkdir -p $O
for i in 1 2; do
  for v in "4 4,1" "1 4,1" "1 1,1" "2 1,1" "2 2,1" "3 4,1"; do
    set -- $v
    timeout -k 10 200 python bench.py --no-legs --no-cpu --fast-side $1 --fast-wpb $2 > $O/fs$1_${2/,/_}_$i.json 2>&1 || exit 1
  done
done
echo done
