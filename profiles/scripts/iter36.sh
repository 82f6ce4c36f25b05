set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5"
GPU_MAX_HW_QUEUES=8 $B > gpurun_out/iter36_a.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 $B --extractors 3 > gpurun_out/iter36_b.log 2>&1 &&
$B > gpurun_out/iter36_c.log 2>&1
