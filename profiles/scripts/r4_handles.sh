# extractor handles per extraction stream 2 vs 3 vs 4 (two extraction streams), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --no-kernel-events"
for i in 1 2; do for h in 2 3 4; do timeout -k 10 200 python bench.py $A --handles-per-stream $h > gpurun_out/hp_${h}_$i.log 2>&1 || exit $?; done; done
