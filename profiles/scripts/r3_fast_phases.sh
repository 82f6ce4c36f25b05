# builds: bash profiles/scripts/build_variant.sh d1 -DORBFE_FAST_DIAG=1 (and d2, d3)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
X="timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq"
$X > gpurun_out/dg_full.log 2>&1 &&
for d in 1 2 3; do ORBFE_LIB=orb_slam2_2021_amd/lib/d$d/liborbfe.so $X > gpurun_out/dg_$d.log 2>&1 || exit 1; done &&
$X > gpurun_out/dg_full2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex k_fast -d gpurun_out/pmcL -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 --seq > gpurun_out/pmcL.log 2>&1 &&
W="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" &&
timeout -k 10 120 python profiles/scripts/match_only.py 50 > gpurun_out/mo.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mo_prof -o run --output-format csv -- python3 profiles/scripts/match_only.py 50 > gpurun_out/mo_prof.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $W --kernel-include-regex 'k_sft|k_vocab' -d gpurun_out/mo_pmc -o run --output-format csv -- python3 profiles/scripts/match_only.py 20 > gpurun_out/mo_pmc.log 2>&1
