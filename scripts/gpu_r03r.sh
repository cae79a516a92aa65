#!/bin/bash
# round 3: the closing build (chains at the default priority): GPU suite, smoke, cfg3 at the driver's setting
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/wl
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/wl/cfg3_driver.json 2> gpurun_out/wl/cfg3_driver.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/wl/cfg3_driver.json')); print('cfg3', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', d['roofline']['frac'], d['cpu_baseline']['value'])"
for I in 2048 4096; do
  timeout -k 10 120 python bench.py --instances $I --steps 20 --warmup 5 --no-cpu > gpurun_out/wl/cfg3_$I.json 2>> gpurun_out/wl/err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/wl/cfg3_$I.json')); print('curve', $I, round(d['value']/1e6,2), 'M/s')"
done
