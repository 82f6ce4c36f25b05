# k_vocab phase costs: ComputeBoW of 32 KeyFrames alone (vocab_only.py) on the default build and on
# the -DORBFE_VOCAB_DIAG=1..5 builds (build_variant.sh vd1..vd5: sorts only / + FeatureVector / all
# but the serial norm / key loads only / empty k_vocab).
# builds: for v in 1 2 3 4 5; do bash profiles/scripts/build_variant.sh vd$v -DORBFE_VOCAB_DIAG=$v; done
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
X="timeout -k 10 120 python profiles/scripts/vocab_only.py 100"
for r in 1; do
  $X > gpurun_out/vph_full_$r.log 2>&1 &&
  for v in 1 2 3 4 5; do ORBFE_LIB=orb_slam2_2021_amd/lib/vd$v/liborbfe.so $X > gpurun_out/vph_${v}_$r.log 2>&1 || exit 1; done
done
