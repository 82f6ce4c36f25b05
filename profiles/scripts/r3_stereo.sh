set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_stereo.py -x -q --timeout 300 --timeout-method thread > gpurun_out/st_test.log 2>&1 &&
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
for r in 1 2; do
  $B > gpurun_out/st_bmatch_$r.log 2>&1 && $B --stereo-on-extract > gpurun_out/st_bext_$r.log 2>&1 || exit 1
done
