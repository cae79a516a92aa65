#!/bin/bash
# GPU parity (pytest -m gpu) then an A/B of environment settings (used through gpurun)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_parity.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_env.sh "$@"
