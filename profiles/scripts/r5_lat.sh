#!/bin/bash
# Round 5: latency schedule on by default for calls of < 8 images -- the whole GPU suite, smoke,
# the C2 A/B, the bench.
set -o pipefail
O=gpurun_out/r5lat
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/scripts/r5_c2_sched.py 3 > $O/c2.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2>&1 || exit 1
echo done
