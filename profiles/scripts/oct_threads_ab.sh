set -o pipefail
mkdir -p gpurun_out/octab
for r in 1 2; do
  for t in 512 1024; do
    ORBFE_OCT_THREADS_SMALL=$t timeout -k 10 200 python -u profiles/scripts/tracking_only.py --no-cpu > gpurun_out/octab/trk_${t}_$r.json 2>/dev/null || exit 1
    python - gpurun_out/octab/trk_${t}_$r.json $t $r >> gpurun_out/octab/summary.txt <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("threads", sys.argv[2], "round", sys.argv[3], "frames/s", d["frames_per_s_one_caller"], "p50_ms", d["latency_ms"]["p50_ms"], "k_octree", d["device_us_per_frame_by_kernel"]["k_octree"], "device_us", d["device_us_per_frame"])
PY
    tail -1 gpurun_out/octab/summary.txt
  done
done
