#!/bin/bash
# round 3: measurement passes (bench + CPU baseline, rocprofv3 stats, FETCH/WRITE/SQ PMC passes) of the
# headline and the workloads the verdict names: cfg3, cfg3 with little-endian seeds, cfg4 N=256, drop64
set -o pipefail
export PYTHONUNBUFFERED=1
bash scripts/gpu_profile.sh cfg3 || exit 1
NAME=cfg3le STEPS=5 bash scripts/gpu_profile.sh cfg3 --seed-order le --cpu-sample 4096 || exit 1
STEPS=3 PSTEPS=1 WARMUP=1 PWARMUP=0 bash scripts/gpu_profile.sh cfg4 --n 256 || exit 1
STEPS=5 PSTEPS=2 WARMUP=1 bash scripts/gpu_profile.sh drop64 --cpu-sample 4096 || exit 1
mkdir -p gpurun_out/prof
bash scripts/gpu_stamps_general.sh > /dev/null 2>&1 || { cat gpurun_out/stamps_general.txt; exit 1; }
cp gpurun_out/stamps_general.txt gpurun_out/prof/
bash scripts/gpu_stamps.sh > /dev/null 2>&1 || { cat gpurun_out/stamps.txt; exit 1; }
cp gpurun_out/stamps.txt gpurun_out/prof/
cat gpurun_out/prof/stamps_general.txt gpurun_out/prof/stamps.txt
