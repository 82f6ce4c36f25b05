#!/bin/bash
# Round 5 final (after the late octree and small-call changes): the whole -m gpu suite, smoke, then
# the bench refresh (full line, rocprofv3 kernel stats of the bench command, a timeline).
set -o pipefail
O=gpurun_out/r5final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
bash profiles/scripts/refresh_profiles.sh bench || exit 1
echo done
