#!/bin/bash
# Round 5 final: the whole -m gpu suite and the smoke entry on the final code.
set -o pipefail
O=gpurun_out/${R5F_OUT:-r5final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
echo done
