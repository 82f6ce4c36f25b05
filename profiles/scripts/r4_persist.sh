# the fixpoint's rounds in one launch with grid barriers (ORBFE_SBP_PERSIST=1): parity first, then
# C5 device time against the default path, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ORBFE_SBP_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py -x -q --timeout 120 --timeout-method thread -k "not settle_kernel_through" > gpurun_out/pe_tests.log 2>&1 &&
for i in 1 2; do
  ORBFE_SBP_PERSIST=1 timeout -k 10 120 python profiles/scripts/c5_only.py 2 --resident --per-kernel > gpurun_out/pe_on_$i.log 2>&1 || exit $?
  timeout -k 10 120 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/pe_off_$i.log 2>&1 || exit $?
done
