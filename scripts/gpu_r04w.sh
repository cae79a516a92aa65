#!/bin/bash
# r04w: drop draws two Philox chains at a time (product) vs one at a time (build/var_seq): parity subset,
# drop64 / cfg2 / cfg4 N=128 / drop64 with the full kernel alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or fullsize" > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for rep in 1 2; do
for v in prod seq; do
  if [ $v = prod ]; then L=consensus-rs_amd/build/libbftsim.so; else L=consensus-rs_amd/build/var_$v/libbftsim.so; fi
  BARGS="--workload drop64 --steps 5 --warmup 1" b drop64_${v}_$rep BFTSIM_LIB=$L
  BARGS="--workload cfg2 --steps 10 --warmup 2" b cfg2_${v}_$rep BFTSIM_LIB=$L
done
done
