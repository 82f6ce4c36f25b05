# The pipeline's cross-stream events: the library's fence-free events (default) vs torch's (system-
# scope write-back on record), interleaved; the C4 proxy with the fence-free events; C3 parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_gather.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ev_tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 120 python bench.py $A > gpurun_out/ev_dev_$r.log 2>&1 &&
  ORBFE_TORCH_EVENTS=1 timeout -k 10 120 python bench.py $A > gpurun_out/ev_torch_$r.log 2>&1 || exit 1
done &&
ORBFE_GPROXY_MODE=pack timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/ev_gp_pack.log 2>&1 &&
timeout -k 10 120 python bench.py $A --gather-proxy 2 > gpurun_out/ev_gp2.log 2>&1 &&
timeout -k 10 120 python bench.py $A --gather-proxy 8 > gpurun_out/ev_gp8.log 2>&1 &&
timeout -k 10 120 python bench.py $A --hw-queues 8 > gpurun_out/ev_hw8.log 2>&1
