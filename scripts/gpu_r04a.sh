#!/bin/bash
# round 4, first pass: GPU suite (new ABI), then cfg3 at the driver's setting and the shard curve
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r04a/gpu_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r04a/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/r04a/cfg3.json 2> gpurun_out/r04a/err || exit 1
for I in 2048 4096; do
  timeout -k 10 120 python bench.py --instances $I --steps 20 --warmup 5 --no-cpu > gpurun_out/r04a/cfg3_$I.json 2>> gpurun_out/r04a/err || exit 1
done
for f in cfg3 cfg3_2048 cfg3_4096; do python3 -c "import json; d=json.load(open('gpurun_out/r04a/$f.json')); print('$f', d['scaling'], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"; done
