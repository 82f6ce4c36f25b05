# kernel timelines (queue ids) of the natively created pipeline streams, 1 and 2 extractors
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R="python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tlA -o run --output-format csv -- $R > gpurun_out/tlA.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tlB -o run --output-format csv -- $R --extractors 2 --pipeline 4 > gpurun_out/tlB.log 2>&1
