# FAST of levels 0..K-1 on the side stream, K = 4 / 5 / 6, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --no-kernel-events"
for i in 1 2; do for k in 4 5 6; do timeout -k 10 200 python bench.py $A --fast-side $k > gpurun_out/fs_${k}_$i.log 2>&1 || exit $?; done; done
