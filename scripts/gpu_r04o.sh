#!/bin/bash
# r04o: Philox rate micro-benchmark; drop64 measurement pass (FAST vs resume kernel times, PMC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04o
timeout -k 10 60 ./tools/philox_rate > gpurun_out/r04o/philox_rate.txt 2>&1 && cat gpurun_out/r04o/philox_rate.txt && \
NAME=drop64 STEPS=5 WARMUP=1 bash scripts/gpu_profile.sh drop64
