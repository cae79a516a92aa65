#!/bin/bash
# round 3: where the split hash pass loses on cfg3 — A/B of the suffix kernel's stream (launch stream vs
# the set's hash stream) against the previous product, and a kernel trace of the product
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace_k
TAG=_k VARS="prod var_sfxhs var_old" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_k -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu > gpurun_out/trace_k/b.json 2> gpurun_out/trace_k/b.err || exit 1
cat gpurun_out/trace_k/run_kernel_stats.csv
