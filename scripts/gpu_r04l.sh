#!/bin/bash
# round 4: GPU suite on the 4-waves build; cfg4 N=128 / N=256 measurement passes (PMC per N); LE occupancy A/B; drop64
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 200 python bench.py --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="--steps 20 --warmup 5" run cfg3
BARGS="--seed-order le --steps 10 --warmup 2" run le_prod
BARGS="--seed-order le --steps 10 --warmup 2" run le_w3 BFTSIM_LIB=consensus-rs_amd/build/var_le3/libbftsim.so
BARGS="--workload drop64 --steps 5 --warmup 1" run drop64
BARGS="--workload cfg2 --steps 10 --warmup 2" run cfg2
NAME=cfg4_n256 STEPS=5 WARMUP=1 PSTEPS=2 PWARMUP=1 bash scripts/gpu_profile.sh cfg4 --n 256 || exit 1
NAME=cfg4_n128 STEPS=5 WARMUP=1 PSTEPS=2 PWARMUP=1 bash scripts/gpu_profile.sh cfg4 --n 128 || exit 1
