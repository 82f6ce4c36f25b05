set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
ORBFE_PYR_HYBRID=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread -k "kitti or pyramid or batch" > gpurun_out/pytest_iter10.log 2>&1 &&
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter10_lv$r.log 2>&1 &&
ORBFE_PYR_HYBRID=1 timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter10_hy$r.log 2>&1 || exit 1
done
ORBFE_PYR_HYBRID=1 timeout -k 10 120 python profiles/scripts/extract_only.py 50 > gpurun_out/iter10_xo.log 2>&1
