#!/bin/bash
# Round 5: DistributeOctTree split into two launches (levels 0-2 at 80 KiB of LDS per block, 3-7 at
# 40 KiB): parity, phase clocks, then the bench with the split (default) and as one launch, interleaved.
set -o pipefail
O=gpurun_out/r5o3
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py -m gpu > $O/tests.log 2>&1 || exit 1
ORBFE_OCT_SPLIT=3 ORBFE_LIB=$L/lib_prof/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu --octree-split 3 > $O/split3_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-legs --no-cpu --octree-split 0 > $O/split0_$i.json 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-legs --no-cpu --octree-split 2 > $O/split2_1.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-legs --no-cpu --octree-split 4 > $O/split4_1.json 2>&1 || exit 1
echo done
