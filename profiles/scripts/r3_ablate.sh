# Ablation (timing only, outputs wrong): the bench line with k_blur skipped (abl1), k_copy0 skipped
# (abl2), matching skipped (--diag-skip-matching), against the full pipeline, interleaved.
# builds: bash profiles/scripts/build_variant.sh abl1 -DORBFE_DIAG_SKIP=1; ... abl2 -DORBFE_DIAG_SKIP=2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
for r in 1 2; do
  $B > gpurun_out/abl_full_$r.log 2>&1 &&
  ORBFE_LIB=orb_slam2_2021_amd/lib/abl1/liborbfe.so $B > gpurun_out/abl_noblur_$r.log 2>&1 &&
  ORBFE_LIB=orb_slam2_2021_amd/lib/abl2/liborbfe.so $B > gpurun_out/abl_nocopy_$r.log 2>&1 &&
  $B --diag-skip-matching > gpurun_out/abl_nomatch_$r.log 2>&1 &&
  $B --no-stereo > gpurun_out/abl_nostereo_$r.log 2>&1 || exit 1
done
