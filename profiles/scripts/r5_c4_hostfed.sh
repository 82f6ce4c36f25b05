#!/bin/bash
# Round 5: the host-fed C3 leg (bench.py --feed host) and C4's rank-0 share measured with the
# one-GPU proxy (--gather-proxy 8: rank 0 receiving 7 payloads per slot), interleaved.
set -o pipefail
mkdir -p gpurun_out/r5c4
O=gpurun_out/r5c4
B="timeout -k 10 240 python bench.py --no-legs --no-cpu --steps 4 --warmup 1 --event-every 1000000"
timeout -k 10 200 python bench.py --feed host --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu \
  > $O/hostfed.json 2> $O/hostfed.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gather.py \
  > $O/gather_tests.log 2>&1 || exit 1
for rep in 1 2; do
  $B > $O/base_$rep.json 2> $O/base_$rep.err || exit 1
  $B --gather-proxy 8 --root-share 1 > $O/p8_full_$rep.json 2> $O/p8_full_$rep.err || exit 1
  $B --gather-proxy 8 > $O/p8_auto_$rep.json 2> $O/p8_auto_$rep.err || exit 1
  NCCL_MAX_NCHANNELS=2 $B --gather-proxy 8 --root-share 1 > $O/p8_ch2_$rep.json 2> $O/p8_ch2_$rep.err || exit 1
done
echo done
