set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5"
$B > gpurun_out/iter24_a.log 2>&1 &&
$B --no-parity --fast-side 2 > gpurun_out/iter24_b.log 2>&1 &&
$B --no-parity --match-normal > gpurun_out/iter24_c.log 2>&1 &&
$B --no-parity > gpurun_out/iter24_d.log 2>&1
