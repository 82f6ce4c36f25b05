set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --match-high > gpurun_out/iter23_a.log 2>&1 &&
$B --extractors 3 --match-inline > gpurun_out/iter23_b.log 2>&1 &&
$B --extractors 1 > gpurun_out/iter23_c.log 2>&1 &&
$B --extractors 3 --match-high > gpurun_out/iter23_d.log 2>&1
