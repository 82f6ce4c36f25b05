#!/bin/bash
# Round 5: small calls' results in one D2H copy -- extraction / host-path / C++ facade tests, the
# C2 A/B, the C2 trace.
set -o pipefail
O=gpurun_out/${R5C2_OUT:-r5c2c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py -m gpu -k "latency_schedule or batch_equals_single or host_batch" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/scripts/r5_c2_sched.py 3 > $O/c2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -- python3 $GRAFT_REPO_ROOT/profiles/scripts/r5_c2_trace.py > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 1
echo done
