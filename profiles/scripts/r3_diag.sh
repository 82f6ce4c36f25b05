# Round 3 first call: baseline bench on this box + the disjoint wait breakdown
# (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY = SQ_WAVE_CYCLES) of k_fast, k_describe, k_sft_nodes.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
SMALL="--no-cpu --no-legs --no-parity --steps 2 --warmup 1 --batches-per-step 16 --probe-subbatches 4"
W="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_r3_0.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $W --kernel-include-regex 'k_fast|k_describe|k_blur|k_resize' -d gpurun_out/pmcW1 -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 > gpurun_out/pmcW1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $W --kernel-include-regex 'k_sft|k_vocab' -d gpurun_out/pmcW2 -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcW2.log 2>&1
