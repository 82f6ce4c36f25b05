# overlapping-extractions experiment: 1 vs 2 vs 3 extractor handles (side work inline for >1)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for e in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors $e > gpurun_out/dual_$e.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 2 --level-launches > gpurun_out/dual_2L.log 2>&1
