set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B > gpurun_out/iter16_a.log 2>&1 &&
$B --pipeline 4 > gpurun_out/iter16_b.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors 2 > gpurun_out/iter16_c.log 2>&1 &&
$B --extractors 2 --pipeline 4 > gpurun_out/iter16_d.log 2>&1 &&
$B --extractors 3 > gpurun_out/iter16_e.log 2>&1 &&
$B --extractors 3 --pipeline 6 > gpurun_out/iter16_f.log 2>&1
