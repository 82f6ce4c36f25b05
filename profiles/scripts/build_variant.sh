# Diagnostic / ablation build of liborbfe.so with extra defines, into orb_slam2_2021_amd/lib/NAME
# (loaded with ORBFE_LIB=orb_slam2_2021_amd/lib/NAME/liborbfe.so; never the default build).
# Usage: bash profiles/scripts/build_variant.sh NAME "-DORBFE_VOCAB_DIAG=1"
set -e
cd "$(dirname "$0")/../../orb_slam2_2021_amd/csrc"
make -s -j8 OBJ=../build/$1 OUT=../lib/$1 EXTRA="$2"
