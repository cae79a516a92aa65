#!/bin/bash
# r04r: little-endian seeds with predictions: launch streams x ring depth (the seed chains and FAST kernels
# of one launch are serial on its launch stream; more streams = more launches' chains in flight)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=8
O=gpurun_out/r04r; mkdir -p $O
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for LS in 2 3 4; do
  for D in 6 8 12; do
    BARGS="--seed-order le --steps 20 --warmup 5 --pipeline-depth $D" b le_ls${LS}_d$D BFTSIM_LAUNCH_STREAMS=$LS
  done
done
for I in 2048 4096; do
  for LS in 2 4; do
    BARGS="--seed-order le --steps 20 --warmup 5 --instances $I --pipeline-depth 16" b le_c${I}_ls$LS BFTSIM_LAUNCH_STREAMS=$LS
  done
done
