set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_register.py tests/test_cpp_facade.py tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hb_test.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 250 --timeout-method thread -k "kf" > gpurun_out/c3kf_test.log 2>&1 &&
timeout -k 10 100 python profiles/scripts/hb_r3.py > gpurun_out/hb1.log 2>&1 &&
ORBFE_HOST_GROUPS=2 timeout -k 10 100 python profiles/scripts/hb_r3.py > gpurun_out/hb2.log 2>&1 &&
ORBFE_HOST_GROUPS=4 timeout -k 10 100 python profiles/scripts/hb_r3.py > gpurun_out/hb4.log 2>&1 &&
ORBFE_HOST_TRACE=1 timeout -k 10 100 python profiles/scripts/hb_r3.py > gpurun_out/hb_trace.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/match_only.py 50 > gpurun_out/mo2.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events > gpurun_out/tl.log 2>&1
