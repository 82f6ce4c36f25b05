# The C4 ingestion proxy with the pipeline's own comm stream, N = 2, 4, 8, beside the 8-queue
# baseline; C5 with the settle path from rounds R0 = 2, 3, 4, 6 and without it.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g3_base.log 2>&1 &&
timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g3_2.log 2>&1 &&
timeout -k 10 120 python bench.py $A --gather-proxy 4 > gpurun_out/g3_4.log 2>&1 &&
timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/g3_8.log 2>&1 &&
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g3_base2.log 2>&1 &&
timeout -k 10 200 python profiles/scripts/c5_only.py 3 --per-kernel --resident > gpurun_out/g3_c5.log 2>&1 &&
for r in 2 3 4 6; do ORBFE_SBP_SETTLE_FROM=$r timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident > gpurun_out/g3_c5_$r.log 2>&1 || exit 1; done &&
ORBFE_SBP_SETTLE=0 timeout -k 10 200 python profiles/scripts/c5_only.py 3 --resident --per-kernel > gpurun_out/g3_c5_old.log 2>&1
