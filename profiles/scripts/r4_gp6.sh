# settle phase clocks at R0 = 2, 4, 8
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 4 6 8 10; do ORBFE_SBP_SETTLE_FROM=$r timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/g6_c5_$r.log 2>&1 || exit 1; done &&
ORBFE_SBP_SETTLE=0 timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/g6_c5_old.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g6_tests.log 2>&1
