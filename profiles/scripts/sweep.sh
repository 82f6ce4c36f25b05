#!/bin/bash
# Interleaved sweep of bench.py argument sets on one box (the multi-variant form of ab.sh):
#   OUT=<name under gpurun_out/>  ROUNDS=<passes, default 2>  BENCH_ARGS=<shared, default "--no-cpu --no-legs">
#   SETS="name1=args1;name2=args2;..."   (an empty args string is the default configuration)
# Each run's JSON line goes to $OUT/<name><round>.json; summary.txt holds value, ms_per_step, parity
# and the per-kernel device time of every run.
set -o pipefail
O=gpurun_out/${OUT:-sweep}
mkdir -p $O
IFS=';' read -ra SETS_ARR <<< "${SETS:-default=}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for kv in "${SETS_ARR[@]}"; do
    name=${kv%%=*}
    args=${kv#*=}
    timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---no-cpu --no-legs} $args > $O/$name$r.json 2> $O/$name$r.err || exit 1
    python - "$O/$name$r.json" "$name$r" >> $O/summary.txt <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d.get("kernels_us_per_subbatch", {})
print(sys.argv[2], round(d["value"]), d["ms_per_step"], "parity", d.get("parity_bit_exact"),
      " ".join(f"{n}={v}" for n, v in sorted(k.items(), key=lambda kv: -kv[1])))
PY
    tail -1 $O/summary.txt
  done
done
echo done
