#!/bin/bash
# round 3 re-entry pass on HEAD: GPU suite + smoke + cfg3 measurement (gpu_full.sh), then the shard
# curve at depth 3 and the other workloads' bench lines
set -o pipefail
export PYTHONUNBUFFERED=1
bash scripts/gpu_full.sh || exit $?
mkdir -p gpurun_out/curve gpurun_out/wl
for I in 2048 4096 8192; do
  timeout -k 10 120 python bench.py --instances $I --steps 20 --warmup 3 --no-cpu > gpurun_out/curve/cfg3_${I}_d3.json 2>> gpurun_out/curve/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/curve/cfg3_${I}_d3.json')); print('curve', $I, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
done
for W in "cfg3 --seed-order le" drop64 cfg2 "cfg4 --n 256" "cfg4 --n 128"; do
  T=$(echo $W | tr -d ' -')
  timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 2 --no-cpu > gpurun_out/wl/$T.json 2>> gpurun_out/wl/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/wl/$T.json')); print('$T', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms/step')"
done
