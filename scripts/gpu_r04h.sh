#!/bin/bash
# round 4: launch streams (consensus round-robin) x ring depth x hardware queues; GPU suite first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for I in 16384 2048 4096; do
  BARGS="--instances $I --pipeline-depth 4 --hw-queues 8" run c${I}_cs0_d4 BFTSIM_LAUNCH_STREAMS=0
  for C in 1 2; do
    for D in 4 5 6; do
      BARGS="--instances $I --pipeline-depth $D --hw-queues 8" run c${I}_cs${C}_d$D BFTSIM_LAUNCH_STREAMS=$C
    done
  done
  BARGS="--instances $I --pipeline-depth 7 --hw-queues 10" run c${I}_cs2_d7_q10 BFTSIM_LAUNCH_STREAMS=2
  BARGS="--instances $I --pipeline-depth 8 --hw-queues 12" run c${I}_cs2_d8_q12 BFTSIM_LAUNCH_STREAMS=2
done
