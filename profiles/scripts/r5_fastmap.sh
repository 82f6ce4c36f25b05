#!/bin/bash
# (ran at commit f55e8c0; the fast modes were removed after the A/B: DESIGN.md section 5)
# k_fast_map + k_fast_cells (fast mode 1): parity, then the full -m gpu suite, then interleaved A/B.
set -o pipefail
O=gpurun_out/r5fm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k fast_map > $O/fm_tests.log 2>&1 || exit 1
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for m in 0 1; do
    timeout -k 10 200 python bench.py --no-legs --no-cpu --fast-mode $m > $O/ab_m${m}_$i.json 2>&1 || exit 1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python bench.py --no-legs --no-cpu --fast-mode 1 --steps 5 > $O/prof1.log 2>&1 || exit 1
echo done
