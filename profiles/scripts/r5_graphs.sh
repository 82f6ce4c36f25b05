#!/bin/bash
# (ran at commit 18192e4, when replay was the library default; replay is opt-in since: --graphs)
# Launch-graph replay: parity (the new test + the extraction / C3 / stereo / C++ facade suites run
# with graphs on), interleaved bench A/B against direct launches, the k_octree phase clocks of the
# profiling builds (-DORBFE_OCT_PROF=1; lib_prof_g16 adds -DORBFE_OCT_GATHER16=1), the gather
# variant's bench A/B (lib_g16), the host-fed leg with 4 and 8 input slots, then the full line.
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_gpu_stereo.py tests/test_cpp_facade.py -m gpu > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/ab_graph_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-legs --no-cpu --no-graphs > $O/ab_direct_$i.json 2>&1 || exit 1
done
ORBFE_LIB=$L/lib_prof/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof.txt 2>&1 || exit 1
ORBFE_LIB=$L/lib_prof_g16/liborbfe.so timeout -k 10 120 python profiles/scripts/r5_octree_prof.py 3 > $O/octree_prof_g16.txt 2>&1 || exit 1
for i in 1 2; do
  ORBFE_LIB=$L/lib_g16/liborbfe.so timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/ab_g16_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/ab_base_$i.json 2>&1 || exit 1
done
for sl in 4 8; do
  timeout -k 10 200 python bench.py --feed host --input-slots $sl --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu --event-every 1000000 > $O/hostfed_$sl.json 2>&1 || exit 1
done
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
echo done
