#!/bin/bash
# round 3: chain priority 3 below 12,000 instances (var_prio) vs var_perm; kernel stats of var_perm on cfg3
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stats_perm
TAG=_prio VARS="var_prio var_perm" WL="cfg3 --instances 2048" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_prio VARS="var_prio var_perm" WL="cfg3 --instances 4096" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_prio VARS="var_prio var_perm" WL="cfg3 --instances 8192" STEPS=20 bash scripts/gpu_abw.sh || exit 1
BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/var_perm/libbftsim.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_perm -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/stats_perm/b.json 2> gpurun_out/stats_perm/b.err || exit 1
cat gpurun_out/stats_perm/run_kernel_stats.csv
