# k_describe's test pattern in LDS as fp16 (25.1 instead of 27.1 KiB per workgroup: three fit beside
# a DistributeOctTree block's 80 KiB) against the float table: parity, then interleaved bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ORBFE_LIB=ab/h16/liborbfe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dh_parity.log 2>&1 || exit $?
A="--no-cpu --no-legs --steps 3"
for i in 1 2 3; do for v in base h16; do
  ORBFE_LIB=ab/$v/liborbfe.so timeout -k 10 200 python bench.py $A > gpurun_out/dh_${v}_$i.log 2>&1 || exit $?
done; done
