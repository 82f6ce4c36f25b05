# The whole bench line (C3 value, host-boundary callers, C5 leg) with 4 (HIP default) vs 8 hardware
# queues, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2"
for r in 1 2; do
  $B --hw-queues 4 > gpurun_out/hwq4_$r.log 2>&1 &&
  $B --hw-queues 8 > gpurun_out/hwq8_$r.log 2>&1 || exit 1
done
