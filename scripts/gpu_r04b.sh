#!/bin/bash
# round 4: GPU suite (new ABI, wave chain, concurrent launches), then the shard curve with A/B of the
# chain kernel (wave / pair) and of concurrent vs serial consensus kernels
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env..., -- bench args
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="" run cfg3_prod
BARGS="" run cfg3_serial BFTSIM_SERIAL_CONSENSUS=1
for I in 2048 4096 8192; do
  BARGS="--instances $I" run c${I}_wave_conc BFTSIM_CHAIN_WAVE_MAX=100000
  BARGS="--instances $I" run c${I}_pair_conc BFTSIM_CHAIN_WAVE_MAX=0
  BARGS="--instances $I" run c${I}_wave_serial BFTSIM_CHAIN_WAVE_MAX=100000 BFTSIM_SERIAL_CONSENSUS=1
  BARGS="--instances $I" run c${I}_pair_serial BFTSIM_CHAIN_WAVE_MAX=0 BFTSIM_SERIAL_CONSENSUS=1
done
BARGS="--instances 2048 --pipeline-depth 4" run c2048_wave_conc_d4 BFTSIM_CHAIN_WAVE_MAX=100000
BARGS="--instances 16384" run c16384_wave_conc BFTSIM_CHAIN_WAVE_MAX=100000
