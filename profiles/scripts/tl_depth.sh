# kernel timelines (with queue ids) of the depth-2 and depth-4 single-handle pipelines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R="python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl2 -o run --output-format csv -- $R > gpurun_out/tl2.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl4 -o run --output-format csv -- $R --pipeline 4 > gpurun_out/tl4.log 2>&1
