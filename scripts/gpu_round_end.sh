#!/bin/bash
# Everything the round-end evidence needs, in one gpurun call: all -m gpu tests, smoke(), the cfg3
# measurement pass (bench + rocprof stats + PMC passes), and the sig / wire measurement passes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_full.sh || exit $?
bash scripts/gpu_sig.sh > gpurun_out/gpu_sig.out 2>&1 || { tail -20 gpurun_out/gpu_sig.out; exit 1; }
bash scripts/gpu_wire.sh > gpurun_out/gpu_wire.out 2>&1 || { tail -20 gpurun_out/gpu_wire.out; exit 1; }
echo "sig:"; grep -E "recoveries/sec" gpurun_out/bench_sig.json | cut -c1-200
echo "wire:"; grep -E "messages/sec" gpurun_out/bench_wire.json | cut -c1-200
