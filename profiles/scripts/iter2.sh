# host boundary iteration: extraction/facade tests, then the bench line with legs (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_cpp_facade.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter2.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --steps 5 > gpurun_out/iter2_bench.log 2>&1
