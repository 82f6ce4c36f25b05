# schedule A/B: FAST of levels 0..K-1 on the side stream
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for k in 3 4 5 6 8; do timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --fast-side $k > gpurun_out/iter5_$k.log 2>&1 || exit 1; done
