# k_octree at 78 instead of 80 KiB of LDS, so that three k_describe workgroups (27.1 KiB each) fit
# beside one octree block: parity, then interleaved bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ORBFE_LIB=ab/o78/liborbfe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 300 --timeout-method thread > gpurun_out/do_parity.log 2>&1 || exit $?
A="--no-cpu --no-legs --steps 3"
for i in 1 2 3; do for v in base o78; do
  ORBFE_LIB=ab/$v/liborbfe.so timeout -k 10 200 python bench.py $A > gpurun_out/do_${v}_$i.log 2>&1 || exit $?
done; done
