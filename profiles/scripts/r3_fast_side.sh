set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
for r in 1 2; do
  for k in ${KS:-2 3 4}; do $B --fast-side $k > gpurun_out/fs_m${k}_$r.log 2>&1 || exit 1; done
done
