set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5"
$B --vocab-inline > gpurun_out/iter25_a.log 2>&1 &&
$B --no-parity --vocab-inline --match-normal > gpurun_out/iter25_b.log 2>&1 &&
$B --no-parity --vocab-inline --extractors 3 --match-inline > gpurun_out/iter25_c.log 2>&1 &&
$B --no-parity > gpurun_out/iter25_d.log 2>&1
