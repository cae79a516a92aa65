#!/bin/bash
# r04u24: the pair Keccak's 24 rounds fully unrolled with constant round constants (build/var_u24) vs the
# round loop with a per-lane round-constant load (product); chain tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04u24; mkdir -p $O
BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/var_u24/libbftsim.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipeline" > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3))"
}
for rep in 1 2; do
for v in prod u24; do
  if [ $v = prod ]; then L=consensus-rs_amd/build/libbftsim.so; else L=consensus-rs_amd/build/var_$v/libbftsim.so; fi
  BARGS="--steps 20 --warmup 5" b cfg3_${v}_$rep BFTSIM_LIB=$L
  BARGS="--steps 20 --warmup 5 --instances 2048" b c2048_${v}_$rep BFTSIM_LIB=$L
  BARGS="--steps 40 --warmup 5 --instances 2048" b c2048k40_${v}_$rep BFTSIM_LIB=$L
  BARGS="--steps 20 --warmup 5 --instances 8192" b c8192_${v}_$rep BFTSIM_LIB=$L
  BARGS="--steps 20 --warmup 5 --seed-order le" b le_${v}_$rep BFTSIM_LIB=$L
done
done
