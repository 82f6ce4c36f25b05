# C5 device time with the settle path from rounds R0 = 2, 3, 4 and without it; matcher tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python profiles/scripts/c5_only.py 3 --per-kernel --resident > gpurun_out/s4_c5.log 2>&1 &&
for r in 2 3 6; do ORBFE_SBP_SETTLE_FROM=$r timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident --per-kernel > gpurun_out/s4_c5_$r.log 2>&1 || exit 1; done &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s4_tests.log 2>&1
