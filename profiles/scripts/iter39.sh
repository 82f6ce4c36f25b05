set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B > gpurun_out/iter39_a.log 2>&1 &&
$B --blur-mode 2 > gpurun_out/iter39_b.log 2>&1 &&
$B --fast-side 2 > gpurun_out/iter39_c.log 2>&1 &&
$B --fast-side 4 > gpurun_out/iter39_d.log 2>&1 &&
$B --pipeline 6 > gpurun_out/iter39_e.log 2>&1 &&
$B > gpurun_out/iter39_f.log 2>&1
