# GPU test suite, then a kernel timeline of the default pipeline (rocprofv3 --kernel-trace, the
# bench's events off) and the extraction alone per kernel (extract_only.py --per-kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq > gpurun_out/r4_alone.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events > gpurun_out/tl.log 2>&1
