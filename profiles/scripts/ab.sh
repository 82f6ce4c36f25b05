#!/bin/bash
# Interleaved A/B on one box: bench.py with two builds of liborbfe.so and/or two argument sets,
# A B A B ... (ROUNDS pairs). Replaces round 5's one-off r5_*.sh launchers.
#   OUT=<name under gpurun_out/>   ROUNDS=<pairs, default 2>
#   LIB_A / LIB_B = liborbfe.so paths (default: the in-tree build; build a variant with
#     make -C orb_slam2_2021_amd/csrc OUT=../lib_b OBJ=../build_b EXTRA=-D...)
#   ARGS_A / ARGS_B = extra bench.py arguments per side; BENCH_ARGS = shared ones
#     (default "--no-cpu --no-legs")
# Each run's JSON line goes to $OUT/<A|B><round>.json; summary.txt holds value, ms_per_step and the
# per-kernel device time of every run.
set -o pipefail
O=gpurun_out/${OUT:-ab}
mkdir -p $O
LIB_DEF=orb_slam2_2021_amd/lib/liborbfe.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in A B; do
    lib=LIB_$v
    args=ARGS_$v
    ORBFE_LIB=${!lib:-$LIB_DEF} timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---no-cpu --no-legs} ${!args} \
      > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python - "$O/$v$r.json" "$v$r" >> $O/summary.txt <<'PY' || exit 1
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
