# multi-rank orchestration rehearsal: 2 ranks on the one GPU, gloo between them, parity per rank
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --rehearse --gpus 2 --steps 1 --warmup 1 --batches-per-step 16 --no-cpu --no-legs > gpurun_out/rehearse.log 2>&1
