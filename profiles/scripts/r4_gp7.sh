# rounds per C5 search, old path and settle from round 8
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ORBFE_SBP_SETTLE=0 timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/g7_old.log 2>&1 &&
ORBFE_SBP_SETTLE_FROM=8 timeout -k 10 200 python profiles/scripts/c5_only.py 2 --resident > gpurun_out/g7_8.log 2>&1
