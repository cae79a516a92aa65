#!/bin/bash
# round 4: resume queue; GPU suite; cfg3 measurement pass (bench + rocprof stats + FETCH/WRITE/SQ PMC)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="" run cfg3
BARGS="--no-pipeline" run cfg3_nopipe
for I in 2048 4096; do BARGS="--instances $I" run c$I; done
BARGS="--workload drop64 --steps 5" run drop64
STEPS=20 WARMUP=5 PSTEPS=5 PWARMUP=2 bash scripts/gpu_profile.sh cfg3 || exit 1
