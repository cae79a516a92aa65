#!/bin/bash
# round 4: finer sweep of launches in flight x hardware queues, and the chain waves' priority
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04d; mkdir -p $O
run() {  # name, env..., (bench args in BARGS)
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for I in 2048 4096; do
  for D in 5 6 7; do
    for Q in 7 8 10; do
      BARGS="--instances $I --pipeline-depth $D --hw-queues $Q" run c${I}_d${D}_q${Q}
    done
  done
  for P in 1 2 3; do
    BARGS="--instances $I --pipeline-depth 6 --hw-queues 8" run c${I}_d6_q8_prio$P BFTSIM_CHAIN_PRIO=$P
  done
done
for rep in 1 2; do
  for D in 3 4 5; do
    BARGS="--pipeline-depth $D --hw-queues 8" run c16384_d${D}_q8_r$rep
  done
  BARGS="--pipeline-depth 3 --hw-queues 4" run c16384_d3_q4_r$rep
done
BARGS="--pipeline-depth 4 --hw-queues 8" run c16384_d4_q8_prio1 BFTSIM_CHAIN_PRIO=1
