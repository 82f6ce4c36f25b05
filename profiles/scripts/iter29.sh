set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --blur-mode 1 > gpurun_out/iter29_a.log 2>&1 &&
$B --blur-mode 0 > gpurun_out/iter29_b.log 2>&1 &&
$B --blur-mode 1 --fast-side 4 > gpurun_out/iter29_c.log 2>&1 &&
$B --blur-mode 0 > gpurun_out/iter29_d.log 2>&1 &&
$B --blur-mode 1 > gpurun_out/iter29_e.log 2>&1 &&
$B --blur-mode 1 --fast-side 5 > gpurun_out/iter29_f.log 2>&1
