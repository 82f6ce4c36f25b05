set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--no-cpu --no-legs --steps 3"
for i in 1 2; do for v in 0 1; do ORBFE_DESC_SIDE=$v timeout -k 10 200 python bench.py $A > gpurun_out/ds_${v}_$i.log 2>&1 || exit $?; done; done
