set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --side-normal > gpurun_out/iter43_a.log 2>&1 &&
$B > gpurun_out/iter43_b.log 2>&1 &&
$B --side-normal > gpurun_out/iter43_c.log 2>&1 &&
$B > gpurun_out/iter43_d.log 2>&1
