# gather proxy: which wait costs (an extraction stream's event; the matching stream at normal priority)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g10_base.log 2>&1 &&
ORBFE_GPROXY_MODE=waitext timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g10_waitext.log 2>&1 &&
ORBFE_MATCH_PRIO=normal timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g10_mnormal.log 2>&1 &&
ORBFE_MATCH_PRIO=normal ORBFE_GPROXY_MODE=waitonly timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g10_mnormal_wait.log 2>&1 &&
ORBFE_MATCH_PRIO=normal timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/g10_mnormal_p8.log 2>&1 &&
ORBFE_GPROXY_MODE=poll timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g10_poll.log 2>&1 &&
ORBFE_GPROXY_MODE=rccl timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g10_rccl2.log 2>&1 &&
ORBFE_GPROXY_MODE=rccl timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/g10_rccl8.log 2>&1
