# k_sft_nodes phase costs: SearchForTriangulation of the 31 KeyFrame pairs alone (match_only.py) on
# the default build and on -DORBFE_SFT_DIAG=1/2 (loads only / + passing sets, no claim rounds;
# wrong matches), plus the ComputeBoW phase builds (r3_vocab_phases.sh).
# builds: bash profiles/scripts/build_variant.sh sd1 -DORBFE_SFT_DIAG=1 (and sd2)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
X="timeout -k 10 120 python profiles/scripts/match_only.py 100"
$X > gpurun_out/sph_full.log 2>&1 &&
for v in 1 2; do ORBFE_LIB=orb_slam2_2021_amd/lib/sd$v/liborbfe.so $X > gpurun_out/sph_$v.log 2>&1 || exit 1; done
