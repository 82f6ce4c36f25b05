# C4 proxy: RCCL on the matching stream vs RCCL on the comm stream ordered by the host (no waits)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g11_base.log 2>&1 &&
for n in 2 4 8; do ORBFE_GPROXY_MODE=rcclhost timeout -k 10 120 python bench.py $A --gather-proxy $n > gpurun_out/g11_host$n.log 2>&1 || exit $?; done &&
ORBFE_GPROXY_MODE=rccl timeout -k 10 120 python bench.py $A --gather-proxy 4 > gpurun_out/g11_rccl4.log 2>&1
