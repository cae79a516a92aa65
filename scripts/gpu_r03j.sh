#!/bin/bash
# round 3: the split block-hash pass (suffix kernel + splice chain): GPU suite, then A/B against the
# previous product library (var_old) on cfg3 and small shards
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
TAG=_split2 VARS="prod var_old" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_split2 VARS="prod var_old" WL="cfg3 --instances 2048" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_split2 VARS="prod var_old" WL=cfg2 STEPS=10 bash scripts/gpu_abw.sh || exit 1
