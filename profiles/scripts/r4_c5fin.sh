# C5 device time without the no-op finish launch; matcher / frustum / keyframe tests
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/cf_1.log 2>&1 &&
timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/cf_2.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py tests/test_gpu_resident_map.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cf_tests.log 2>&1
