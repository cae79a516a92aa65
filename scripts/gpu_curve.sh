#!/bin/bash
# one-GPU shard-size curve of cfg3 at several pipeline depths (through gpurun), plus the pipeline tests
set -o pipefail
mkdir -p gpurun_out/curve
export PYTHONUNBUFFERED=1
cat /sys/fs/cgroup/cpu.max > gpurun_out/curve/cpu_max.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/curve/tests.log 2>&1 || { tail -20 gpurun_out/curve/tests.log; exit 1; }
tail -1 gpurun_out/curve/tests.log
for I in 2048 4096 8192 16384; do for D in 2 3 4 6; do
  timeout -k 10 120 python bench.py --instances $I --pipeline-depth $D --steps 20 --warmup 3 --no-cpu > gpurun_out/curve/cfg3_${I}_d$D.json 2>> gpurun_out/curve/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/curve/cfg3_${I}_d$D.json')); print('curve', $I, 'depth', $D, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
done; done
