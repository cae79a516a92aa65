#!/bin/bash
# r04u: Philox keys from opaque scalars (no SGPR spills into VGPR lanes in the general kernels' drop loop):
# GPU suite, then drop64 / cfg2 / cfg4 N=256 and N=128 / cfg3 / cfg3-LE bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() {
  local name=$1; shift
  env BFTSIM_TESTING=1 "$@" timeout -k 10 300 python bench.py --no-cpu $BARGS > $O/$name.json 2> $O/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="--workload drop64 --steps 5 --warmup 1" b drop64
BARGS="--workload cfg2 --steps 10 --warmup 2" b cfg2
BARGS="--workload cfg4 --n 256 --steps 5 --warmup 1" b cfg4_n256
BARGS="--workload cfg4 --n 128 --steps 5 --warmup 1" b cfg4_n128
BARGS="--steps 20 --warmup 5" b cfg3
BARGS="--seed-order le --steps 20 --warmup 5" b cfg3_le
