set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --extra-streams 1 > gpurun_out/iter15_a.log 2>&1 &&
$B --extra-streams 2 > gpurun_out/iter15_b.log 2>&1 &&
$B --extra-streams 3 > gpurun_out/iter15_c.log 2>&1 &&
$B --pipeline 4 --extra-streams 2 > gpurun_out/iter15_d.log 2>&1 &&
$B --extractors 2 --shared-side --pipeline 4 --extra-streams 1 > gpurun_out/iter15_e.log 2>&1
