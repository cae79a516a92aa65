#!/bin/bash
# round 3: GPU parity of the product on the segment-kernel cases, then occupancy A/Bs
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r03f
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "256 or 128 or 200 or 100 or 65" --timeout 200 --timeout-method thread > gpurun_out/r03f/parity_prod.log 2>&1 || { tail -30 gpurun_out/r03f/parity_prod.log; exit 1; }
tail -1 gpurun_out/r03f/parity_prod.log
TAG=_f256 VARS="prod" WL="cfg4 --n 256" STEPS=3 bash scripts/gpu_abw.sh || exit 1
TAG=_f128 VARS="prod var_b128_2" WL="cfg4 --n 128" STEPS=3 bash scripts/gpu_abw.sh || exit 1
TAG=_fw4 VARS="prod var_w4" WL=drop64 bash scripts/gpu_abw.sh || exit 1
TAG=_fw4 VARS="prod var_w4" WL=cfg2 bash scripts/gpu_abw.sh || exit 1
