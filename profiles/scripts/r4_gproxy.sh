# C4 proxy (RCCL self pairs on the matching stream), N = 2 / 4 / 8, gathered every 1 or 4
# sub-batches, beside the 8-queue baseline; then the gather test file
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/gp_base.log 2>&1 &&
for n in 2 4 8; do for k in 1 4; do timeout -k 10 120 python bench.py $A --gather-proxy $n --gather-every $k > gpurun_out/gp_${n}_$k.log 2>&1 || exit $?; done; done &&
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/gp_base2.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_gather.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gp_tests.log 2>&1
