set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter8.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 > gpurun_out/iter8_a.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter8_b.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 50 > gpurun_out/iter8_xo.log 2>&1 &&
bash profiles/scripts/pmc_bench_valu.sh
