#!/bin/bash
# Round 5: host-side phases of the C2 call (ORBFE_HOST_TRACE, one image, 60 calls per schedule).
set -o pipefail
O=gpurun_out/r5c2h
mkdir -p $O
ORBFE_HOST_TRACE=1 timeout -k 10 120 python -u profiles/scripts/r5_c2_trace.py > $O/run.log 2> $O/trace.log || exit 1
echo done
