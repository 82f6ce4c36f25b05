set -o pipefail
mkdir -p gpurun_out/r5sweep
timeout -k 10 120 python profiles/scripts/c5_only.py 4 --resident > gpurun_out/r5sweep/c5_q.txt 2>&1
