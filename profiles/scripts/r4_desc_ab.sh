# k_describe without the LDS tables (pattern and masks through the vector L1, 5 waves / SIMD) vs
# the committed kernel, interleaved; extraction parity of B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3"
for i in 1 2; do for v in A B; do ORBFE_LIB=$PWD/ab/lib$v.so timeout -k 10 200 python bench.py $A > gpurun_out/dab_${v}_$i.log 2>&1 || exit $?; done; done &&
ORBFE_LIB=$PWD/ab/libB.so timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dab_tests.log 2>&1
