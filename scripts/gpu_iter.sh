#!/bin/bash
# one iteration on the GPU box: consensus/hash kernel ms (unpipelined), the bench line, the GPU suite
# usage: scripts/gpu_iter.sh [pytest -k expression]
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/diag_kms.py 21 0 21:le > gpurun_out/kms.txt 2>&1 && cat gpurun_out/kms.txt && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/bench20.json 2> gpurun_out/bench20.err && \
python3 -c "import json; d=json.load(open('gpurun_out/bench20.json')); print('bench', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel_ms'])" && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
exit $rc
