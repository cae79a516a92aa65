#!/bin/bash
# Copy the summaries of a scripts/gpu_profile.sh run (gpurun_out/prof) into profiles/<round>/ (tracked).
set -e
R=${1:-r01}
D=profiles/$R
mkdir -p $D/pmc
cp gpurun_out/prof/stats/run_kernel_stats.csv $D/kernel_stats.csv
cp gpurun_out/prof/stats/run_kernel_trace.csv $D/kernel_trace.csv
cp gpurun_out/prof/pmc_summary.json $D/pmc_summary.json
for p in fetch write sq; do cp gpurun_out/prof/$p/run_counter_collection.csv $D/pmc/${p}_counter_collection.csv; done
cp gpurun_out/bench.json $D/bench.json
cp gpurun_out/host_cpu.txt $D/host_cpu.txt
[ -f gpurun_out/gpu_parity.log ] && tail -3 gpurun_out/gpu_parity.log > $D/gpu_parity_tail.txt || true
echo "saved to $D"
