#!/bin/bash
# r04s: little-endian seeds with predictions: seeded launch streams 4 / 6 / 8 x GPU_MAX_HW_QUEUES, shard sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04s; mkdir -p $O
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for LS in 4 6 8; do
  for Q in 8 12 16; do
    BARGS="--seed-order le --steps 20 --warmup 5 --hw-queues $Q" b le_ls${LS}_q$Q BFTSIM_LAUNCH_STREAMS_SEEDED=$LS
  done
done
for I in 2048 4096 8192; do
  for LS in 4 8; do
    BARGS="--seed-order le --steps 20 --warmup 5 --instances $I --hw-queues 16" b le_c${I}_ls$LS BFTSIM_LAUNCH_STREAMS_SEEDED=$LS
  done
done
BARGS="--steps 20 --warmup 5" b cfg3
