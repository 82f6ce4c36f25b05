set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
$B --diag-skip-matching > gpurun_out/iter35_a.log 2>&1 &&
$B --diag-skip-matching --extractors 3 --match-inline > gpurun_out/iter35_b.log 2>&1 &&
$B > gpurun_out/iter35_c.log 2>&1
