# GaussianBlur fused into k_describe (lib/fused, -DORBFE_FUSED_BLUR=1) against the in-tree library:
# extraction alone and the bench line interleaved, then the fused build's bench parity (keypoints,
# descriptors, BowVector, FeatureVector, match12 vs the oracle chain).
# build: bash profiles/scripts/build_variant.sh fused -DORBFE_FUSED_BLUR=1
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-fu}
ALT=orb_slam2_2021_amd/lib/fused/liborbfe.so
X="timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq"
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
ORBFE_LIB=$ALT timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 1 --warmup 1 > gpurun_out/${T}_parity.log 2>&1 &&
$X > gpurun_out/${T}_xold1.log 2>&1 && ORBFE_LIB=$ALT $X > gpurun_out/${T}_xnew1.log 2>&1 &&
$B > gpurun_out/${T}_bold1.log 2>&1 && ORBFE_LIB=$ALT $B > gpurun_out/${T}_bnew1.log 2>&1 &&
$B > gpurun_out/${T}_bold2.log 2>&1 && ORBFE_LIB=$ALT $B > gpurun_out/${T}_bnew2.log 2>&1
