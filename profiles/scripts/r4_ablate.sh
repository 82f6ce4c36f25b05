# Round-4 ablations, interleaved: default, no ComputeStereoMatches, extraction only, FAST of levels
# 0..3 on the side stream (the bench's short form, no legs / CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
for r in 1 2; do
  timeout -k 10 120 python bench.py $A > gpurun_out/ab_def_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --no-stereo > gpurun_out/ab_nost_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --diag-skip-matching > gpurun_out/ab_extr_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --fast-side 4 > gpurun_out/ab_fs4_$r.log 2>&1 || exit 1
done
