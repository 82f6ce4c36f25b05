# Round-4 measurement call: the bench line (no legs, no CPU) and rocprofv3 --kernel-trace --stats
# of the same command, so the line's dispatch-bound kernel times can be checked against rocprof's.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ARGS="--no-cpu --no-legs --steps 3 --warmup 1"
timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r4_prof.log 2>&1
