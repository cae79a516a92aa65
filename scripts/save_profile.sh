#!/bin/bash
# Copy the summaries of scripts/gpu_profile.sh runs (gpurun_out/prof/<workload>) into profiles/<round>/
# (tracked): the headline (cfg3) at profiles/<round>/, every other workload at profiles/<round>/<workload>/.
# usage: scripts/save_profile.sh <round> <workload>...
set -e
RND=$1; shift
for W in "$@"; do
  S=gpurun_out/prof/$W
  [ "$W" = cfg3 ] && D=profiles/$RND || D=profiles/$RND/$W
  mkdir -p $D/pmc
  cp $S/stats/run_kernel_stats.csv $D/kernel_stats.csv
  cp $S/pmc_summary.json $D/pmc_summary.json
  for p in fetch write sq; do cp $S/$p/run_counter_collection.csv $D/pmc/${p}_counter_collection.csv; done
  cp $S/bench.json $D/bench.json
  cp $S/host_cpu.txt $D/host_cpu.txt
  echo "saved $W to $D"
done
