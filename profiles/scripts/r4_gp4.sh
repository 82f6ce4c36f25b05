# Which part of the --gather-proxy path costs: pack only, events only, copies on the matching
# stream, no release wait; then the settle sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/g4_base.log 2>&1 &&
for mode in packonly evonly same norelease torch; do ORBFE_GPROXY_MODE=$mode timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/g4_$mode.log 2>&1 || exit 1; done &&
bash profiles/scripts/r4_settle.sh
