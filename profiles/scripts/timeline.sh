# kernel timeline of a short bench run (for the critical-path analysis)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events "$@" > gpurun_out/tl.log 2>&1
