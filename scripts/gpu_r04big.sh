#!/bin/bash
# r04big: chain batch x ring depth at 16,384 per GPU (the N = 1 headline), three repetitions each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04big; mkdir -p $O
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3))"
}
for rep in 1 2 3; do
  for BD in "2 6" "4 8" "3 6" "4 12"; do
    set -- $BD
    BARGS="--hash-batch $1 --pipeline-depth $2 --steps 20 --warmup 5" b c16384_b$1_d$2_$rep
  done
done
