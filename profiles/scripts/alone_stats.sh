# per-kernel durations with one sub-batch in flight (one handle, one output set): the kernels'
# own times: no other handle, no side-stream overlap, no matching beside the extraction
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/alone -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 128 --probe-subbatches 4 --no-kernel-events --extractors 1 --pipeline 1 --inline-side > gpurun_out/alone.log 2>&1
