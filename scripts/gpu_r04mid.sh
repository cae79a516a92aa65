#!/bin/bash
# r04mid: chain batch x ring depth at the N = 2 and N = 4 strong-scaling shards (8,192 and 4,096 per GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04mid; mkdir -p $O
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3))"
}
for I in 8192 4096 12288; do
  for BD in "2 6" "4 8" "4 12" "6 12" "8 16" "3 8"; do
    set -- $BD
    BARGS="--instances $I --hash-batch $1 --pipeline-depth $2 --steps 20 --warmup 5" b c${I}_b$1_d$2
  done
done
