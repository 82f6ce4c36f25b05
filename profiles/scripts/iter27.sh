set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3"
$B > gpurun_out/iter27_a.log 2>&1 &&
$B --extractors 1 > gpurun_out/iter27_b.log 2>&1
