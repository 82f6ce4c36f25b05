# The default bench line with several builds of liborbfe.so (orb_slam2_2021_amd/lib/NAME, "" = the
# in-tree default), interleaved twice. Usage: bash r3_libs.sh tag "" NAME1 NAME2 ... [-- bench flags]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1 $*"
for r in 1 2; do
  i=0
  for Lb in "${LIBS[@]}"; do
    if [ -z "$Lb" ]; then $B > gpurun_out/${T}_m${i}_${r}.log 2>&1 || exit 1
    else ORBFE_LIB=orb_slam2_2021_amd/lib/$Lb/liborbfe.so $B > gpurun_out/${T}_m${i}_${r}.log 2>&1 || exit 1; fi
    i=$((i + 1))
  done
done
