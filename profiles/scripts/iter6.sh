set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
python -c "import torch; print(torch.cuda.Stream.priority_range())" > gpurun_out/prio.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter6_a.log 2>&1 &&
ORBFE_EXTRACT_PRIORITY=-1 timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter6_b.log 2>&1 &&
ORBFE_EXTRACT_PRIORITY=-2 timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter6_c.log 2>&1
