#!/bin/bash
# Round 5: wave_child_split inlined (it was an out-of-line call whose LDS pointers became flat
# accesses): parity (extraction, C3, golden), phase clocks, per-pass clocks, the bench.
set -o pipefail
O=gpurun_out/r5o7
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || exit 1
ORBFE_LIB=$L/lib_prof/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof.txt 2>&1 || exit 1
for k in 2 3; do
  ORBFE_OCT_PROF_PASS=$k ORBFE_LIB=$L/lib_pp$k/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/pass$k.txt 2>&1 || exit 1
done
timeout -k 10 300 python bench.py > $O/bench_1.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/bench_2.json 2>&1 || exit 1
echo done
