#!/bin/bash
# round 3: branch-free v_perm prefix encoder in the hash chains (var_perm) against the split pass (var_split)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/var_perm/libbftsim.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_perm.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_perm.log; [ $rc -eq 0 ] || exit $rc
TAG=_perm VARS="var_perm var_split" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_perm VARS="var_perm var_split" WL="cfg3 --instances 2048" STEPS=20 bash scripts/gpu_abw.sh || exit 1
