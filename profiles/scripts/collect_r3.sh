# Copy the round-3 measurement summaries from gpurun_out/ (refresh_profiles.sh and the experiment
# scripts) into profiles/ (run locally after the GPU calls).
set -e
cd "$(dirname "$0")/../.."
tail -n 1 gpurun_out/bench_full.log > profiles/r3_bench.json
cp gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_c5.json profiles/
python3 profiles/scripts/valu_summary.py gpurun_out/pmcWait/run_counter_collection.csv > profiles/r3_valu.txt
cp gpurun_out/prof/run_kernel_stats.csv profiles/r3_kernel_stats.csv
{ echo "# wave-time breakdown, bench (contended): rocprofv3 --pmc of bench.py (refresh_profiles.sh, pmcWait)";
  python3 profiles/pmc_waits.py gpurun_out/pmcWait/run_counter_collection.csv;
  echo; echo "# alone: one 64-image extraction at a time (extract_only.py --seq, pmcAlone)";
  python3 profiles/pmc_waits.py gpurun_out/pmcAlone/run_counter_collection.csv; } > profiles/r3_pmc_waits.txt
python3 profiles/scripts/timeline_view.py gpurun_out/tl > profiles/r3_timeline.txt
