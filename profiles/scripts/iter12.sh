set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 5 --extractors 2 --shared-side --pipeline 4 > gpurun_out/iter12_a.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 2 --shared-side --pipeline 6 > gpurun_out/iter12_b.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 2 --shared-side --pipeline 8 > gpurun_out/iter12_c.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 3 --shared-side --pipeline 6 > gpurun_out/iter12_d.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --extractors 2 --pipeline 4 > gpurun_out/iter12_e.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 5 --pipeline 4 > gpurun_out/iter12_f.log 2>&1
