set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5"
$B --blur-mode 2 > gpurun_out/iter28_a.log 2>&1 &&
$B --blur-mode 1 > gpurun_out/iter28_b.log 2>&1 &&
$B --no-parity > gpurun_out/iter28_c.log 2>&1 &&
$B --no-parity --blur-mode 2 --fast-side 2 > gpurun_out/iter28_d.log 2>&1
