set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --streams-first"
$B > gpurun_out/iter13_a.log 2>&1 &&
$B --pipeline 4 > gpurun_out/iter13_b.log 2>&1 &&
$B --extractors 2 --shared-side --pipeline 3 > gpurun_out/iter13_c.log 2>&1 &&
$B --extractors 2 --shared-side --pipeline 4 > gpurun_out/iter13_d.log 2>&1 &&
$B --extractors 2 --shared-side --pipeline 6 > gpurun_out/iter13_e.log 2>&1 &&
$B --extractors 3 --shared-side --pipeline 4 > gpurun_out/iter13_f.log 2>&1
