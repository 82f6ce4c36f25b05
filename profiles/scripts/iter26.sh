set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --pipeline 6 > gpurun_out/iter26_a.log 2>&1 &&
$B --pipeline 8 > gpurun_out/iter26_b.log 2>&1 &&
$B --input-batches 16 > gpurun_out/iter26_c.log 2>&1 &&
$B --batches-per-step 512 --steps 10 > gpurun_out/iter26_d.log 2>&1
