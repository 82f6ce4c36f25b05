# the round's final evidence: the whole GPU suite, then the bench line, its profiled twin and the timeline
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 &&
bash profiles/scripts/refresh_profiles.sh bench
