#!/bin/bash
# Round 5: k_octree's thread-serial / wavefront split threshold OCT_SMALL (48 default; 32 / 64 / 96
# as profiling builds): the phase clocks of each, interleaved twice.
set -o pipefail
O=gpurun_out/r5os
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
for r in 1 2; do
  for v in prof os32 os64 os96; do
    ORBFE_LIB=$L/lib_$v/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/${v}_$r.txt 2>&1 || exit 1
  done
done
echo done
