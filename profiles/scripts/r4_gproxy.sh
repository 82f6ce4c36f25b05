# C4 rank-0 ingestion proxy on one GPU (bench.py --gather-proxy N), interleaved with the default
# line at the same hardware-queue setting (8, as with N > 1).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
for r in 1 2; do
  timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/gp_base_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/gp_2_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --gather-proxy 4 > gpurun_out/gp_4_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/gp_8_$r.log 2>&1 || exit 1
done
