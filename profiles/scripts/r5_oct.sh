#!/bin/bash
# Round 5: k_octree's initial-node loops bounded by the wave's key rows; the phase clocks of the
# profiling build (orb_slam2_2021_amd/lib_prof, -DORBFE_OCT_PROF=1) with marks inside the first pass
# and refinement round; the bench line twice; the host-fed leg with 4 and 8 input slots.
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py -m gpu > $O/tests.log 2>&1 || exit 1
ORBFE_LIB=$L/lib_prof/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/bench_$i.json 2>&1 || exit 1
done
for sl in 4 8; do
  timeout -k 10 200 python bench.py --feed host --input-slots $sl --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu --event-every 1000000 > $O/hostfed_$sl.json 2>&1 || exit 1
done
echo done
