# k_fast check: extraction parity tests, per-kernel times of one 64-image extraction, and the
# k_fast instruction-mix counters (one PMC pass).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_c3.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel > gpurun_out/xo.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_fast -d gpurun_out/pmcA -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcA.log 2>&1
