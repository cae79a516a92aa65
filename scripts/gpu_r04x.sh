#!/bin/bash
# r04x: the general body's fused block phase and composed canonical view (S >= 64): the whole GPU suite,
# then cfg4 N=256 / N=128, cfg2, drop64, cfg3 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r04x}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="--workload cfg4 --n 256 --steps 5 --warmup 1" b cfg4_n256
BARGS="--workload cfg4 --n 128 --steps 5 --warmup 1" b cfg4_n128
BARGS="--workload cfg2 --steps 10 --warmup 2" b cfg2
BARGS="--workload drop64 --steps 5 --warmup 1" b drop64
BARGS="--steps 20 --warmup 5" b cfg3
