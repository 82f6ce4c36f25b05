set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c3.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_kf.log 2>&1
