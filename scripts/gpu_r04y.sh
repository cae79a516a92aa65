#!/bin/bash
# r04y: measurement passes of cfg4 N=256 / N=128 after the general-body fusions (bench + rocprof stats + PMC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
STEPS=5 WARMUP=1 NAME=r04y/cfg4_n256 bash scripts/gpu_profile.sh cfg4 --n 256 || exit 1
STEPS=5 WARMUP=1 NAME=r04y/cfg4_n128 bash scripts/gpu_profile.sh cfg4 --n 128 || exit 1
