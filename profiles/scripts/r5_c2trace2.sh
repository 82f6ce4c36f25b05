#!/bin/bash
# Round 5: kernel + memory-copy trace of the C2 call after the small-call changes.
set -o pipefail
O=gpurun_out/r5c2t2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -- python3 $GRAFT_REPO_ROOT/profiles/scripts/r5_c2_trace.py > $GRAFT_REPO_ROOT/$O/run.log 2>&1 || exit 1
echo done
