# schedule iteration: extraction/C3/stereo tests, bench (no legs), lone-extraction timing
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter4.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter4_bench.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 50 > gpurun_out/iter4_xo.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel >> gpurun_out/iter4_xo.log 2>&1
