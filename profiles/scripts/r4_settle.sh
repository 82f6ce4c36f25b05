# The SearchByProjection settle path: the matcher parity tests, then C5's device time per search
# with and without it (ORBFE_SBP_SETTLE=0: one launch per round), per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py tests/test_gpu_resident_map.py -x -q --timeout 200 --timeout-method thread > gpurun_out/st_tests.log 2>&1 &&
timeout -k 10 200 python profiles/scripts/c5_only.py 3 --per-kernel --resident > gpurun_out/st_c5_new.log 2>&1 &&
ORBFE_SBP_SETTLE=0 timeout -k 10 200 python profiles/scripts/c5_only.py 3 --per-kernel --resident > gpurun_out/st_c5_old.log 2>&1 &&
timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident > gpurun_out/st_c5_new_plain.log 2>&1 &&
timeout -k 10 300 python profiles/scripts/tracking_only.py --no-cpu > gpurun_out/st_trk.log 2>&1
