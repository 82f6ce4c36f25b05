#!/bin/bash
# Round 5: the host-fed C3 leg (bench.py --feed host): input ring of 8 / 16 slots, and the H2D copies
# by blit kernels instead of the SDMA engines (HSA_ENABLE_SDMA=0), interleaved.
set -o pipefail
O=gpurun_out/r5hf
mkdir -p $O
HF="--feed host --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu --event-every 1000000"
for i in 1 2; do
  timeout -k 10 200 python bench.py $HF > $O/sdma_$i.json 2>&1 || exit 1
  HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench.py $HF > $O/blit_$i.json 2>&1 || exit 1
done
timeout -k 10 200 python bench.py $HF --input-slots 16 > $O/sdma_s16.json 2>&1 || exit 1
HSA_ENABLE_SDMA=0 timeout -k 10 200 python profiles/scripts/h2d_bw.py > $O/h2d_bw_blit.txt 2>&1 || exit 1
timeout -k 10 200 python profiles/scripts/h2d_bw.py > $O/h2d_bw_sdma.txt 2>&1 || exit 1
echo done
