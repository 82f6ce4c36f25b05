set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5"
$B --vocab-side > gpurun_out/iter31_a.log 2>&1 &&
$B --no-parity > gpurun_out/iter31_b.log 2>&1 &&
$B --no-parity --vocab-side --fast-side 2 > gpurun_out/iter31_c.log 2>&1 &&
$B --no-parity --vocab-side > gpurun_out/iter31_d.log 2>&1
