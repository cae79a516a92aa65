#!/bin/bash
# GPU parity run (used through gpurun): pytest -m gpu with its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu 2>&1 | tee gpurun_out/gpu_parity.log
