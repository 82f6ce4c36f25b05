# k_pyramid counters (two passes) over a short extraction run
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex k_pyramid -d gpurun_out/pmcP1 -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcP1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --kernel-include-regex k_pyramid -d gpurun_out/pmcP2 -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcP2.log 2>&1
