set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 python profiles/scripts/hb_sweep.py > gpurun_out/hb.log 2>&1 &&
ORBFE_HOST_TWO_H2D=1 timeout -k 10 60 python profiles/scripts/hb_sweep.py >> gpurun_out/hb.log 2>&1 &&
ORBFE_HOST_GROUPS=2 timeout -k 10 60 python profiles/scripts/hb_sweep.py >> gpurun_out/hb.log 2>&1 &&
ORBFE_HOST_TRACE=1 timeout -k 10 60 python profiles/scripts/hb_sweep.py > gpurun_out/hb_trace.log 2>&1 &&
ORBFE_HOST_TRACE=1 ORBFE_HOST_TWO_H2D=1 timeout -k 10 60 python profiles/scripts/hb_sweep.py > gpurun_out/hb_trace2.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_cpp_facade.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_hb.log 2>&1
