# Regenerates the committed measurement artefacts in two GPU calls (run from the repo root):
#   bash profiles/scripts/refresh_profiles.sh bench   -- the full bench line, rocprofv3 kernel
#        stats of the bench command (its own JSON line is in prof.log: the line's ktimer and the
#        trace see the same run), and a kernel timeline
#   bash profiles/scripts/refresh_profiles.sh pmc     -- FETCH_SIZE / WRITE_SIZE passes (HBM traffic
#        per kernel) of the bench and of the C5 search, the wave-time breakdown, contended and alone
# Outputs under gpurun_out/; the PMC traffic summaries are also copied to profiles/ on the box, so a
# bench line of a later call reports them.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
SMALL="--no-cpu --no-legs --no-parity --steps 2 --warmup 1 --batches-per-step 16 --probe-subbatches 4"
W="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
case "$1" in
bench)
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --steps 3 > gpurun_out/prof.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --no-cpu --no-legs --no-parity --steps 1 --warmup 1 --batches-per-step 64 --probe-subbatches 4 --no-kernel-events > gpurun_out/tl.log 2>&1
;;
pmc)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcF.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcW.log 2>&1 &&
python3 profiles/pmc_summary.py gpurun_out/pmcF/run_counter_collection.csv gpurun_out/pmcW/run_counter_collection.csv gpurun_out/pmc_traffic.json > /dev/null && cp gpurun_out/pmc_traffic.json profiles/ &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c5F -o run --output-format csv -- python3 profiles/scripts/c5_only.py 5 > gpurun_out/c5F.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c5W -o run --output-format csv -- python3 profiles/scripts/c5_only.py 5 > gpurun_out/c5W.log 2>&1 &&
python3 profiles/pmc_c5_summary.py gpurun_out/c5F/run_counter_collection.csv gpurun_out/c5W/run_counter_collection.csv 81 gpurun_out/pmc_traffic_c5.json > /dev/null && cp gpurun_out/pmc_traffic_c5.json profiles/ &&
timeout -s KILL 120 rocprofv3 --pmc $W -d gpurun_out/pmcWait -o run --output-format csv -- python3 bench.py $SMALL > gpurun_out/pmcWait.log 2>&1 &&
python3 profiles/pmc_waits.py gpurun_out/pmcWait/run_counter_collection.csv --json gpurun_out/pmc_waits.json --workload '{"cols": 1241, "rows": 376, "batch": 32, "pairs": "kf", "stereo": true}' > gpurun_out/pmc_waits_contended.txt && cp gpurun_out/pmc_waits.json profiles/ &&
timeout -s KILL 90 rocprofv3 --pmc $W --kernel-include-regex 'k_' -d gpurun_out/pmcAlone -o run --output-format csv -- python3 profiles/scripts/extract_only.py 5 --seq > gpurun_out/pmcAlone.log 2>&1
;;
*) echo "usage: refresh_profiles.sh bench|pmc"; exit 2;;
esac
