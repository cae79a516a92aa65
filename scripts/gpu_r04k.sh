#!/bin/bash
# round 4: FAST kernel occupancy A/B (6 waves/SIMD with spills vs 5 vs 4 without), cfg3 + small shards
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04k; mkdir -p $O
run() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for r in 1 2; do
  for V in prod var_w5 var_w4; do
    L=""; [ $V != prod ] && L="BFTSIM_LIB=consensus-rs_amd/build/$V/libbftsim.so"
    BARGS="--no-pipeline" run ${V}_nopipe_r$r $L
    BARGS="" run ${V}_cfg3_r$r $L
    BARGS="--instances 2048" run ${V}_c2048_r$r $L
  done
done
