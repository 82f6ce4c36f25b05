# HBM traffic of the matching kernels alone (match_only.py): FETCH_SIZE and WRITE_SIZE passes for the
# in-tree build and lib/$1
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/smF0 -o run --output-format csv -- python3 profiles/scripts/match_only.py 10 > gpurun_out/smF0.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/$1/liborbfe.so timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/smF1 -o run --output-format csv -- python3 profiles/scripts/match_only.py 10 > gpurun_out/smF1.log 2>&1 &&
timeout -k 10 120 python profiles/scripts/match_only.py 100 > gpurun_out/sm_t0.log 2>&1 &&
ORBFE_LIB=orb_slam2_2021_amd/lib/$1/liborbfe.so timeout -k 10 120 python profiles/scripts/match_only.py 100 > gpurun_out/sm_t1.log 2>&1
