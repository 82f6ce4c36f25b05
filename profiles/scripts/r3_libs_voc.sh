# ComputeBoW alone (vocab_only.py) with several builds (orb_slam2_2021_amd/lib/NAME, "" = in-tree)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=$1; shift
i=0
for Lb in "$@"; do
  if [ -z "$Lb" ]; then timeout -k 10 120 python profiles/scripts/vocab_only.py 100 > gpurun_out/${T}_v${i}.log 2>&1 || exit 1
  else ORBFE_LIB=orb_slam2_2021_amd/lib/$Lb/liborbfe.so timeout -k 10 120 python profiles/scripts/vocab_only.py 100 > gpurun_out/${T}_v${i}.log 2>&1 || exit 1; fi
  i=$((i + 1))
done
