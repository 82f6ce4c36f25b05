set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --fast-side 1 > gpurun_out/iter21_1.log 2>&1 &&
$B --fast-side 2 > gpurun_out/iter21_2.log 2>&1 &&
$B > gpurun_out/iter21_3.log 2>&1 &&
$B --fast-side 5 > gpurun_out/iter21_5.log 2>&1 &&
$B --fast-side 8 > gpurun_out/iter21_8.log 2>&1
