# interleaved A/B of the in-tree library and orb_slam2_2021_amd/lib/alt (same bench flags)
# (build the other variant first: make -C orb_slam2_2021_amd/csrc OUT=../lib/alt OBJ=../build_alt)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 $*"
$B > gpurun_out/ab_new1.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/alt/liborbfe.so $B > gpurun_out/ab_old1.log 2>&1 &&
$B > gpurun_out/ab_new2.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/alt/liborbfe.so $B > gpurun_out/ab_old2.log 2>&1
