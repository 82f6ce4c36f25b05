# SearchLocalPoints (C5) with sparse rounds (default) vs every query every round (ORBFE_SBP_DENSE=1):
# the SBP tests, device time per search, and FETCH_SIZE of the SBP kernels
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sbp_test.log 2>&1 &&
timeout -k 10 200 python profiles/scripts/c5_only.py 5 > gpurun_out/sbp_t0.log 2>&1 &&
ORBFE_SBP_DENSE=1 timeout -k 10 200 python profiles/scripts/c5_only.py 5 > gpurun_out/sbp_t1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/sbpF0 -o run --output-format csv -- python3 profiles/scripts/c5_only.py 2 > gpurun_out/sbpF0.log 2>&1 &&
ORBFE_SBP_DENSE=1 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/sbpF1 -o run --output-format csv -- python3 profiles/scripts/c5_only.py 2 > gpurun_out/sbpF1.log 2>&1
