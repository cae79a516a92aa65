#!/bin/bash
# all GPU parity tests, then the cfg3 bench line without the CPU leg (through gpurun)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_parity.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(round(d['value']/1e6,1), 'M instance-rounds/s', d['roofline']['kernel_ms'])"
