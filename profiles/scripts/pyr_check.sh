# pyramid check: extraction parity tests and per-kernel times of one 64-image extraction, both
# pyramid paths
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pyr.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel > gpurun_out/xo.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --levels > gpurun_out/xo_levels.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 50 > gpurun_out/xo_plain.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 50 --levels >> gpurun_out/xo_plain.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/xo_trace -o run --output-format csv -- python3 profiles/scripts/extract_only.py 10 > gpurun_out/xo_trace.log 2>&1
