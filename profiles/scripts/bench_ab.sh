# A/B of the C3 bench line: default vs --level-launches (no CPU baseline, no legs, no parity)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/ab_tiled.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --level-launches > gpurun_out/ab_levels.log 2>&1
