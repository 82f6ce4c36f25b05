# rocprofv3 kernel stats of the matching chain alone (match_only.py: ComputeBoW + SearchForTriangulation
# repeated on one sub-batch), default build and the -DORBFE_SFT_DIAG phase builds sd1..sd5
# (build_variant.sh sdN -DORBFE_SFT_DIAG=N; wrong match12, read by nothing but the count here)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sft_prof -o run --output-format csv -- python3 profiles/scripts/match_only.py 100 > gpurun_out/sft_prof.log 2>&1 &&
for v in 1 2; do
  ORBFE_LIB=orb_slam2_2021_amd/lib/sd$v/liborbfe.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sft_prof$v -o run --output-format csv -- python3 profiles/scripts/match_only.py 100 > gpurun_out/sft_prof$v.log 2>&1 || exit 1
done
