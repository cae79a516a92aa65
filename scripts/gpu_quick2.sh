#!/bin/bash
# selected GPU tests (argument: pytest -k expression or files), then a short cfg3 bench line
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest $1 -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/quick.log 2>&1
rc=$?
tail -3 gpurun_out/quick.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/quick.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(round(d['value']/1e6,1), 'M instance-rounds/s', d['config']['stats_allreduce'], d['config']['safety_violations'])"
