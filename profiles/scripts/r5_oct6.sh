#!/bin/bash
# Round 5: k_octree per-full-pass clocks (profiling builds with -DORBFE_OCT_PROF_PASS=1,2,3).
set -o pipefail
O=gpurun_out/r5o6
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
for k in 2 3; do
  ORBFE_OCT_PROF_PASS=$k ORBFE_LIB=$L/lib_pp$k/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/pass$k.txt 2>&1 || exit 1
done
echo done
