#!/bin/bash
# round 2, session A: full GPU parity (incl. little-endian seeds, ABI lifecycle), section stamps of the
# FAST kernel, bench lines for big- and little-endian seeds
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_parity.log | head -20; exit $rc; }
bash scripts/gpu_stamps.sh || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_be.json 2> gpurun_out/bench_be.err || exit $?
cat gpurun_out/bench_be.json | cut -c1-400
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --seed-order le > gpurun_out/bench_le.json 2> gpurun_out/bench_le.err || exit $?
cat gpurun_out/bench_le.json | cut -c1-400
