set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors 2 --match-inline > gpurun_out/iter17_c.log 2>&1 &&
$B --extractors 3 --match-inline > gpurun_out/iter17_d.log 2>&1 &&
$B --extractors 2 --match-inline --pipeline 4 > gpurun_out/iter17_e.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors 2 --pipeline 4 > gpurun_out/iter17_f.log 2>&1
