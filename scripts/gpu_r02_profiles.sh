#!/bin/bash
# round 2 measurement pass (through gpurun): every consensus workload's bench line + rocprof + PMC, and
# the one-GPU shard-size curve of cfg3 (the strong-scaling shards of 16,384 over 1/2/4/8 GPUs)
set -o pipefail
mkdir -p gpurun_out/prof gpurun_out/curve
export PYTHONUNBUFFERED=1
bash scripts/gpu_profile.sh cfg3 || exit $?
for I in 2048 4096 8192 16384; do
  timeout -k 10 120 python bench.py --instances $I --steps 20 --warmup 3 --no-cpu > gpurun_out/curve/cfg3_$I.json 2>> gpurun_out/curve/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/curve/cfg3_$I.json')); print('curve', $I, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', d['roofline']['kernel_ms'])"
done
bash scripts/gpu_profile.sh cfg2 || exit $?
bash scripts/gpu_profile.sh drop64 || exit $?
STEPS=3 PSTEPS=1 bash scripts/gpu_profile.sh cfg4 --n 256 || exit $?
STEPS=1 WARMUP=0 PSTEPS=1 PWARMUP=0 bash scripts/gpu_profile.sh cfg5 || exit $?
