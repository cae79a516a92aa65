#!/bin/bash
# A/B of environment settings on the cfg3 bench (used through gpurun): each "VAR=value" (or "-")
# runs twice; e.g. gpu_ab_env.sh - BFTSIM_FAST=0
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/ab.txt
for v in "$@"; do
  for rep in 1 2; do
    if [ "$v" = "-" ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || exit 1
    python - "$v" "$rep" >> gpurun_out/ab.txt <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_one.json"))
print(sys.argv[1], "rep" + sys.argv[2], round(d["value"] / 1e6, 2), "M/s", d["roofline"]["kernel_ms"],
      d["config"]["committed_heights_per_step"])
PY
  done
done
cat gpurun_out/ab.txt
