set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_c3.py > gpurun_out/pytest_iter18.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/iter18_bench.log 2>&1
