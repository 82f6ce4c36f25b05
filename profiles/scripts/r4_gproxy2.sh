# Which part of --gather-proxy costs: the pack alone, the copies as torch (blit) copies, the copies
# as CU kernel copies (ORBFE_GPROXY_MODE), at N = 2 and 8, beside the 8-queue baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g2_base.log 2>&1 &&
ORBFE_GPROXY_MODE=pack timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g2_pack.log 2>&1 &&
ORBFE_GPROXY_MODE=kcopy timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g2_kcopy2.log 2>&1 &&
ORBFE_GPROXY_MODE=kcopy timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/g2_kcopy8.log 2>&1 &&
ORBFE_GPROXY_MODE=torch timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g2_torch2.log 2>&1 &&
timeout -k 10 120 python bench.py $A > gpurun_out/g2_base4.log 2>&1
