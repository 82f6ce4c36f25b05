# kernel timelines of the default pipeline with two builds (in-tree, lib/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R="timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -o run"
A="python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 256 --probe-subbatches 4 --no-kernel-events"
$R -d gpurun_out/tlA -- $A > gpurun_out/tlA.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/$1/liborbfe.so $R -d gpurun_out/tlB -- $A > gpurun_out/tlB.log 2>&1
