#!/bin/bash
# Round 5: a second full bench line on the final code (run-to-run range of the quoted figures).
set -o pipefail
O=gpurun_out/r5fb2
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo done
