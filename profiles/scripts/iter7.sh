set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter7_a.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --defer-matching > gpurun_out/iter7_b.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --defer-matching --pipeline 4 > gpurun_out/iter7_c.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-legs --gpus 2 --rehearse --steps 2 --batches-per-step 32 --defer-matching > gpurun_out/iter7_r.log 2>&1
ORBFE_EARLY_F0_WAIT=1 timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter7_e.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread -k "host_batch or batch_equals" > gpurun_out/pytest_iter7.log 2>&1
