#!/bin/bash
# Round 5: OCT_SMALL 64 (default now) vs 48 -- the whole GPU suite on 64, then the bench A/B
# interleaved (48 from a build with -DOCT_SMALL=48 through ORBFE_LIB), then the full line.
set -o pipefail
O=gpurun_out/r5os64
mkdir -p $O
L=$PWD/orb_slam2_2021_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/b64_$r.json 2>&1 || exit 1
  ORBFE_LIB=$L/lib_os48/liborbfe.so timeout -k 10 200 python bench.py --no-legs --no-cpu > $O/b48_$r.json 2>&1 || exit 1
done
timeout -k 10 600 python bench.py > $O/bench_full.json 2>&1 || exit 1
echo done
