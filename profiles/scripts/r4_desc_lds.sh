# k_describe LDS variants (round 4 A/B): computed IC_Angle masks (no s_mom), and the blurred
# window in two 21-row passes; parity of each, then interleaved bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in mom half hbp; do
  ORBFE_LIB=ab/$v/liborbfe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dl_parity_$v.log 2>&1 || exit $?
done
A="--no-cpu --no-legs --steps 3"
for i in 1 2; do for v in base mom half hbp; do
  ORBFE_LIB=ab/$v/liborbfe.so timeout -k 10 200 python bench.py $A > gpurun_out/dl_${v}_$i.log 2>&1 || exit $?
done; done
