#!/bin/bash
# r04q: little-endian seeds with the seed chain's predicted blocks — LE parity (GPU suite cases, full size),
# bench LE with predictions on / off; drop64 with the resume kernel at 4 waves/SIMD (build/var_r4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=8
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="--seed-order le --steps 20 --warmup 5" b le_spec
BARGS="--seed-order le --steps 20 --warmup 5" b le_nospec BFTSIM_SEED_SPEC=0
BARGS="--steps 20 --warmup 5" b cfg3
BARGS="--workload drop64 --steps 5 --warmup 1" b drop64_r4 BFTSIM_LIB=consensus-rs_amd/build/var_r4/libbftsim.so
