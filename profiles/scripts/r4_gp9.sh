# wait-source experiments for the gather proxy (RCCL on the matching stream last), then the whole
# GPU test suite unless an experiment hung or crashed
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash profiles/scripts/r4_gp8.sh; st=$?
echo "experiments exit $st" > gpurun_out/g10_status.log
case $st in 124|137|134|139) exit $st;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g10_tests.log 2>&1
