# Tracking's per-frame sequence with the settle kernel from round 2, 4 and 8 (default)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 8 2 4 8; do ORBFE_SBP_SETTLE_FROM=$r timeout -k 10 200 python profiles/scripts/tracking_only.py --no-cpu > gpurun_out/ts_$r.log 2>&1 || exit $?; done
