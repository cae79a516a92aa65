#!/bin/bash
# round 4: shard curve vs pipeline depth and hardware queues (concurrent launches, lane-pair chains)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04c; mkdir -p $O
run() {  # name, env..., (bench args in BARGS)
  local name=$1; shift
  env BFTSIM_TESTING=1 BFTSIM_CHAIN_WAVE_MAX=0 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for I in 2048 4096; do
  for D in 3 4 6 8; do
    BARGS="--instances $I --pipeline-depth $D" run c${I}_d${D}_q4 GPU_MAX_HW_QUEUES=4
    BARGS="--instances $I --pipeline-depth $D" run c${I}_d${D}_q8 GPU_MAX_HW_QUEUES=8
  done
  BARGS="--instances $I --pipeline-depth 8" run c${I}_d8_q12 GPU_MAX_HW_QUEUES=12
done
for D in 3 4 6; do
  BARGS="--pipeline-depth $D" run c16384_d${D}_q8 GPU_MAX_HW_QUEUES=8
done
BARGS="--pipeline-depth 4" run c16384_d4_q4 GPU_MAX_HW_QUEUES=4
