# Interleaved A/B of the tracking leg alone (profiles/scripts/tracking_only.py) with an environment
# switch: ENV_A / ENV_B (e.g. ENV_B=ORBFE_SBP_FETCH_SYNC=1), ROUNDS pairs; summary under gpurun_out/trkab.
set -o pipefail
mkdir -p gpurun_out/trkab
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    e=ENV_$v
    env ${!e:-X_NONE=1} timeout -k 10 200 python -u profiles/scripts/tracking_only.py --no-cpu > gpurun_out/trkab/$v$r.json 2>/dev/null || exit 1
    python - gpurun_out/trkab/$v$r.json $v$r >> gpurun_out/trkab/summary.txt <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "frames/s", d["frames_per_s_one_caller"], "p50_ms", d["latency_ms"]["p50_ms"], "device_us", d["device_us_per_frame"])
PY
    tail -1 gpurun_out/trkab/summary.txt
  done
done
