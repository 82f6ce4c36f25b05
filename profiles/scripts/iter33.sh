set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_stereo.py > gpurun_out/pytest_iter33.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter33_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/alone -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 128 --probe-subbatches 4 --no-kernel-events --extractors 1 --pipeline 1 --inline-side > gpurun_out/alone.log 2>&1
