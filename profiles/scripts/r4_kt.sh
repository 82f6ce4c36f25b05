# Every kernel timed on the timed region's event sub-batches: the value with and without the
# events, and the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3"
timeout -k 10 200 python bench.py $A > gpurun_out/kt_ev1.log 2>&1 &&
timeout -k 10 200 python bench.py $A --no-kernel-events > gpurun_out/kt_noev.log 2>&1 &&
timeout -k 10 200 python bench.py $A > gpurun_out/kt_ev2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktprof -o run --output-format csv -- python3 bench.py $A > gpurun_out/kt_prof.log 2>&1
