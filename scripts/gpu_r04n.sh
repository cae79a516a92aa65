#!/bin/bash
# round 4: deep rings (up to 16 sets) x chain batches (up to 8 launches) x hash streams; GPU suite first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for I in 2048 4096 16384; do
  for B in 4 8; do
    for D in 8 12 16; do
      for HS in 2 3; do
        BARGS="--instances $I --hash-batch $B --pipeline-depth $D" run c${I}_b${B}_d${D}_hs$HS BFTSIM_HASH_STREAMS=$HS
      done
    done
  done
done
