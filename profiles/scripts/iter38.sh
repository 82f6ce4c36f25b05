set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --extractors 3 --inline-side > gpurun_out/iter38_a.log 2>&1 &&
$B --extractors 2 --inline-side > gpurun_out/iter38_b.log 2>&1 &&
$B --extractors 4 --inline-side > gpurun_out/iter38_c.log 2>&1 &&
$B --extractors 3 --inline-side --pipeline 9 > gpurun_out/iter38_d.log 2>&1
