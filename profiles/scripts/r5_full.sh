#!/bin/bash
# The whole -m gpu suite, then the default bench line.
set -o pipefail
O=gpurun_out/r5full
mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo done
