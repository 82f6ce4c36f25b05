#!/bin/bash
# Round 5: k_octree's initial nodes and first full pass as one counting sort: parity (extraction,
# C3, golden), phase clocks of the profiling build, the bench twice.
set -o pipefail
O=gpurun_out/r5o4
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || exit 1
ORBFE_LIB=$L/lib_prof/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/bench_$i.json 2>&1 || exit 1
done
echo done
