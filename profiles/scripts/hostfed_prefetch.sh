# Host-fed C3 leg (bench.py --feed host, as legs.c3_host_fed runs it) with the copy stream fed in several ways
# arms (ARMS: bench options, space-separated, an arm's own options joined by commas, e.g. "--copies-ahead=3 --copy-thread"), ROUNDS interleaved rounds; summary under gpurun_out/hfpf/summary.txt.
set -o pipefail
mkdir -p gpurun_out/hfpf
for r in $(seq 1 ${ROUNDS:-2}); do
  for a in ${ARMS:---copies-ahead=0 --copies-ahead=3 --copy-thread}; do
    timeout -k 10 200 python -u bench.py --feed host --steps 3 --warmup 1 --batches-per-step 256 --no-legs --no-cpu \
      --event-every 1000000 ${a//,/ } ${EXTRA} > gpurun_out/hfpf/a${a//[^a-z0-9]/}.r$r.log 2>&1 || exit 1
    python - gpurun_out/hfpf/a${a//[^a-z0-9]/}.r$r.log "$a round=$r" >> gpurun_out/hfpf/summary.txt <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "value", d["value"], "h2d_GBps", d["feed"]["h2d_GBps"], "slots", d["feed"]["device_slots"],
      "ahead", d["feed"]["copies_ahead"], "parity", d.get("parity_bit_exact"))
PY
    tail -1 gpurun_out/hfpf/summary.txt
  done
done
