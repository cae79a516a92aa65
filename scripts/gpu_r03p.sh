#!/bin/bash
# round 3: the suffix rows by a thread per instance on the hash stream from 6,144 instances per launch
# (prod) vs all on the launch stream (var_m0, the previous product) vs the parallel form on the hash
# stream (var_sfx1); GPU suite on the product first
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
TAG=_p VARS="prod var_m0 var_sfx1" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_p VARS="prod var_m0" WL="cfg3 --instances 8192" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_p VARS="prod var_m0" WL=cfg2 STEPS=10 bash scripts/gpu_abw.sh || exit 1
