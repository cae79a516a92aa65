#!/bin/bash
# round 3: RoundChangeSet capacity test on the GPU, then the split hash pass (transposed suffix rows)
# against the previous product (var_old)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "capacity" --timeout 120 --timeout-method thread > gpurun_out/gpu_rcs.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_rcs.log; [ $rc -eq 0 ] || exit $rc
TAG=_split3 VARS="prod var_old" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_split3 VARS="prod var_old" WL="cfg3 --instances 2048" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_split3 VARS="prod var_old" WL="cfg3 --instances 4096" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_split3 VARS="prod var_old" WL=cfg2 STEPS=10 bash scripts/gpu_abw.sh || exit 1
