# k_describe phase costs (diagnostic builds -DORBFE_DESC_DIAG=1: window loads only, 2: + IC_Angle,
# fastAtan2, cos/sin; wrong descriptors) against the full kernel, extraction alone.
# builds: bash profiles/scripts/build_variant.sh dd1 -DORBFE_DESC_DIAG=1; ... dd2 -DORBFE_DESC_DIAG=2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
X="timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq"
$X > gpurun_out/ddg_full.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/dd1/liborbfe.so $X > gpurun_out/ddg_1.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/dd2/liborbfe.so $X > gpurun_out/ddg_2.log 2>&1 &&
$X > gpurun_out/ddg_full2.log 2>&1
