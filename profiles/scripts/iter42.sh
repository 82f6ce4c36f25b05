set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py > gpurun_out/pytest_iter42.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter42_a.log 2>&1
