set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel > gpurun_out/xo.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_fast -d gpurun_out/pmcA -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcA.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex k_fast -d gpurun_out/pmcB -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcB.log 2>&1
