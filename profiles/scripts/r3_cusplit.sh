# Extractor handles on disjoint CU sets (hipExtStreamCreateWithCUMask) vs the shared-CU default.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
for r in 1 2; do
  $B > gpurun_out/cus_base_$r.log 2>&1 &&
  $B --cu-split 1 > gpurun_out/cus_c1_$r.log 2>&1 &&
  $B --cu-split 2 > gpurun_out/cus_c2_$r.log 2>&1 &&
  $B --cu-split 2 --extractors 3 > gpurun_out/cus_c2e3_$r.log 2>&1 &&
  $B --cu-split 2 --extractors 4 > gpurun_out/cus_c2e4_$r.log 2>&1 || exit 1
done
