#!/bin/bash
# The whole -m gpu suite, then the driver's smoke entry, then (optionally) the default bench line.
#   OUT=<name under gpurun_out/>  BENCH=1 to add `python bench.py` (its JSON line -> bench.json)
#   TESTS="tests/test_x.py ..." to run a subset instead of the whole suite
set -o pipefail
O=gpurun_out/${OUT:-suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || exit 1
fi
echo done
