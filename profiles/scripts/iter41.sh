set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 1"
$B > gpurun_out/iter41_a.log 2>&1 &&
$B --copy0-main > gpurun_out/iter41_b.log 2>&1 &&
$B > gpurun_out/iter41_c.log 2>&1 &&
$B --copy0-main > gpurun_out/iter41_d.log 2>&1
