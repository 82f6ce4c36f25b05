#!/bin/bash
# Round 5: small-call latency work -- one D2H copy of a small call's results, the deferred side
# enqueue (A/B), ComputeStereoMatches enqueued behind the stereo Frame's extraction: tests, the C2
# A/B, the bench (c2_latency / adapter / tracking legs).
set -o pipefail
O=gpurun_out/r5c2e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_cpp_facade.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/scripts/r5_c2_sched.py 3 > $O/c2.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2>&1 || exit 1
echo done
