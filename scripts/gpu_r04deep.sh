#!/bin/bash
# r04deep: rings up to 32 sets x chain batches up to 16 launches at small shards (the strong-scaling shards)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04deep; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipeline" > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3))"
}
for I in 2048 4096 8192; do
  for BD in "8 16" "12 24" "16 32"; do
    set -- $BD
    BARGS="--instances $I --hash-batch $1 --pipeline-depth $2 --steps 20 --warmup 5" b c${I}_b$1_d$2
  done
done
BARGS="--instances 2048 --hash-batch 16 --pipeline-depth 32 --steps 40 --warmup 5" b c2048_b16_d32_s40
