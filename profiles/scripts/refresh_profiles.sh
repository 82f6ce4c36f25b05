# One GPU call that regenerates the committed measurement artefacts (run from the repo root):
# the full bench line, rocprofv3 kernel stats of the bench, FETCH_SIZE / WRITE_SIZE PMC passes
# (HBM traffic per kernel), per-kernel VALU/SALU instruction totals and the k_fast counters.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
SMALL="--no-cpu --no-legs --no-parity --steps 2 --warmup 1 --batches-per-step 16 --probe-subbatches 4"
timeout -k 10 500 python bench.py > gpurun_out/bench_full.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --steps 3 > gpurun_out/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcF.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcW.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcV -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcV.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_fast -d gpurun_out/pmcA -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcA.log 2>&1
