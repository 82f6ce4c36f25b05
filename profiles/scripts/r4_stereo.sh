# bench after the stereo row ordering, and the PMC traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3"
timeout -k 10 200 python bench.py $A > gpurun_out/so_1.log 2>&1 &&
timeout -k 10 200 python bench.py $A > gpurun_out/so_2.log 2>&1 &&
bash profiles/scripts/refresh_profiles.sh pmc
