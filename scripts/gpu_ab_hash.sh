#!/bin/bash
# parity (pytest -m gpu) then bench A/B of the block-hash kernels (used through gpurun)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_pair.json 2> gpurun_out/bench.err && \
BFTSIM_HASH=lane timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_lane.json 2>> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/gpu_parity.log
cat gpurun_out/bench_pair.json gpurun_out/bench_lane.json
exit $rc
