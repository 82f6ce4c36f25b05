# Round-4 pipeline-shape A/B, interleaved (short bench form): handles per extraction stream, and
# ComputeBoW on the shared side stream.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3 --warmup 1 --no-parity"
for r in 1 2; do
  timeout -k 10 120 python bench.py $A > gpurun_out/md_def_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --handles-per-stream 3 > gpurun_out/md_h3_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --handles-per-stream 4 > gpurun_out/md_h4_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --vocab-side > gpurun_out/md_vs_$r.log 2>&1 &&
  timeout -k 10 120 python bench.py $A --vocab-side --handles-per-stream 3 > gpurun_out/md_vsh3_$r.log 2>&1 || exit 1
done
