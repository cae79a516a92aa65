#!/bin/bash
# round 3 measurement pass after the secp256k1 change: sig pass (parity, mad peak, throughput, rocprof),
# real-crypto mode (tests + crypto bench line), headline cfg3 profile (bench + CPU baseline, rocprof, PMC)
set -o pipefail
export PYTHONUNBUFFERED=1
bash scripts/gpu_sig.sh > gpurun_out/gpu_sig.out 2>&1 || { tail -20 gpurun_out/gpu_sig.out; exit 1; }
grep -E "recoveries" gpurun_out/bench_sig.json | cut -c1-300
bash scripts/gpu_crypto.sh > gpurun_out/gpu_crypto.out 2>&1 || { tail -20 gpurun_out/gpu_crypto.out; exit 1; }
tail -4 gpurun_out/gpu_crypto.out | cut -c1-300
bash scripts/gpu_profile.sh cfg3 || exit 1
