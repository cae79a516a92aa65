#!/bin/bash
# A/B of the two hash post-pass kernels + parity (used through gpurun)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_parity.log 2>&1 && \
BFTSIM_HASH=coop timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cfg3 or cfg2 or n4" > gpurun_out/gpu_parity_coop.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_lane.json 2> gpurun_out/bench.err && \
BFTSIM_HASH=coop timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_coop.json 2>> gpurun_out/bench.err
rc=$?
tail -2 gpurun_out/gpu_parity.log; tail -2 gpurun_out/gpu_parity_coop.log
python -c "
import json
for f in ('lane','coop'):
    d=json.load(open('gpurun_out/bench_%s.json'%f)); print(f, d['value'], d['roofline']['kernel_ms'])
"
exit $rc
