set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 > gpurun_out/iter11_1.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors 2 --shared-side > gpurun_out/iter11_2s.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 2 --shared-side --pipeline 4 > gpurun_out/iter11_2s4.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 3 --shared-side > gpurun_out/iter11_3s.log 2>&1
