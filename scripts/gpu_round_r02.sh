#!/bin/bash
# round-2 end pass: the whole GPU suite, then one bench line per workload (saved under gpurun_out/wl/)
set -o pipefail
mkdir -p gpurun_out/wl
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_suite.log | head -20; exit $rc; }
B="timeout -k 10 400 python bench.py"
$B --workload cfg2 --steps 10 --warmup 2 --no-cpu > gpurun_out/wl/cfg2.json 2>/dev/null && \
$B --workload cfg2 --byz 1 --steps 10 --warmup 2 --no-cpu > gpurun_out/wl/cfg2b.json 2>/dev/null && \
$B --workload drop64 --steps 5 --warmup 1 --no-cpu > gpurun_out/wl/drop64.json 2>/dev/null && \
$B --workload cfg4 --n 256 --steps 3 --warmup 1 --no-cpu > gpurun_out/wl/cfg4.json 2>/dev/null && \
$B --workload cfg5 --steps 1 --warmup 0 --no-cpu > gpurun_out/wl/cfg5.json 2>/dev/null && \
$B --workload cfg5 --byz 2 --steps 1 --warmup 0 --no-cpu > gpurun_out/wl/cfg5b.json 2>/dev/null && \
$B --seed-order le --steps 3 --warmup 1 --no-cpu > gpurun_out/wl/cfg3le.json 2>/dev/null && \
$B --workload crypto --steps 3 --warmup 1 > gpurun_out/wl/crypto.json 2>/dev/null
rc=$?
for f in gpurun_out/wl/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', '%.3e' % d['value'], d['config']['workload'][:70])"; done
exit $rc
