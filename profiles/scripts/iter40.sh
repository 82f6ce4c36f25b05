set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_gpu_stereo.py > gpurun_out/pytest_iter40.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter40_a.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --copy0-main > gpurun_out/iter40_b.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter40_c.log 2>&1
