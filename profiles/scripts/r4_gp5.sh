# The gather proxy with a high-priority comm stream (the matching stream's priority); C5 settle
# sweep after the settle kernel's LDS / load-batching changes; matcher tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g5_base.log 2>&1 &&
ORBFE_COMM_PRIO=high timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g5_h2.log 2>&1 &&
ORBFE_COMM_PRIO=high timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/g5_h8.log 2>&1 &&
ORBFE_COMM_PRIO=high ORBFE_GPROXY_MODE=evonly timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g5_hev.log 2>&1 &&
for r in 2 4 6 8; do ORBFE_SBP_SETTLE_FROM=$r timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident --per-kernel > gpurun_out/g5_c5_$r.log 2>&1 || exit 1; done &&
ORBFE_SBP_SETTLE=0 timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident --per-kernel > gpurun_out/g5_c5_old.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_frustum.py tests/test_gpu_keyframe.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g5_tests.log 2>&1
