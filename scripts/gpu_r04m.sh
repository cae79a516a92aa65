#!/bin/bash
# round 4 measurement pass: cfg3 at the driver's setting (bench + rocprof stats + FETCH/WRITE/SQ PMC + kernel trace),
# the 2,048-per-GPU strong-scaling shard the same way
set -o pipefail
export PYTHONUNBUFFERED=1
STEPS=20 WARMUP=5 PSTEPS=5 PWARMUP=2 bash scripts/gpu_profile.sh cfg3 || exit 1
NAME=cfg3_2048 STEPS=20 WARMUP=5 PSTEPS=5 PWARMUP=2 bash scripts/gpu_profile.sh cfg3 --instances 2048 || exit 1
NAME=cfg3_4096 STEPS=20 WARMUP=5 PSTEPS=5 PWARMUP=2 bash scripts/gpu_profile.sh cfg3 --instances 4096 || exit 1
python3 scripts/trace_overlap.py gpurun_out/prof/cfg3/stats/run_kernel_trace.csv --last 20
python3 scripts/trace_overlap.py gpurun_out/prof/cfg3_2048/stats/run_kernel_trace.csv --last 20
