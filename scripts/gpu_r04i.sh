#!/bin/bash
# round 4: batched chain kernels (hash_batch launches per kernel) x ring depth x hash streams; GPU suite first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for I in 16384 2048 4096; do
  for B in 1 2 4; do
    for D in 4 6 8; do
      BARGS="--instances $I --pipeline-depth $D" run c${I}_b${B}_d$D BFTSIM_HASH_BATCH=$B
    done
  done
  BARGS="--instances $I --pipeline-depth 8" run c${I}_b4_d8_hs1 BFTSIM_HASH_BATCH=4 BFTSIM_HASH_STREAMS=1
  BARGS="--instances $I --pipeline-depth 8" run c${I}_b4_d8_hs3 BFTSIM_HASH_BATCH=4 BFTSIM_HASH_STREAMS=3
  BARGS="--instances $I --pipeline-depth 8" run c${I}_b3_d8 BFTSIM_HASH_BATCH=3
done
