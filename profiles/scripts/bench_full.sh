set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/bench_full.log 2>&1
