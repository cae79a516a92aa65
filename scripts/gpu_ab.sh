#!/bin/bash
# A/B timing of library variants (consensus-rs_amd/build/variants/*.so) in ONE box session:
# a quick parity check, then bench.py (no CPU leg) per variant. Used through gpurun.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/ab.txt
for lib in consensus-rs_amd/build/variants/*.so; do
  name=$(basename "$lib" .so)
  BFTSIM_LIB="$PWD/$lib" timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cfg3 or cfg2 or cfg4-n64 or n10" > "gpurun_out/ab_parity_$name.log" 2>&1 || { echo "$name parity FAILED" >> gpurun_out/ab.txt; exit 1; }
  for rep in 1 2; do
    BFTSIM_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > "gpurun_out/ab_$name.json" 2> "gpurun_out/ab_$name.err" || { echo "$name bench FAILED" >> gpurun_out/ab.txt; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', 'rep$rep', round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_ms'])" >> gpurun_out/ab.txt
  done
done
cat gpurun_out/ab.txt
