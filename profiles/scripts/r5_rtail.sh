#!/bin/bash
# (ran with a k_resize_tail kernel that was removed after this A/B)
# Round 5: pyramid levels 4-7 in one k_resize_tail launch -- parity (extraction, C3), then the bench
# with the tail (default) and with a launch per level, interleaved, and the C2 / tracking legs.
set -o pipefail
O=gpurun_out/r5rt
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py -m gpu > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/tail4_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-legs --no-cpu --resize-tail 0 > $O/tail0_$i.json 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-legs --no-cpu --resize-tail 3 > $O/tail3_1.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-legs --no-cpu --resize-tail 5 > $O/tail5_1.json 2>&1 || exit 1
echo done
