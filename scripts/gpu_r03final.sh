#!/bin/bash
# round 3 closing pass on HEAD: GPU suite + smoke + cfg3 measurement (bench + rocprof + PMC), the
# driver's 20-step cfg3 line, the hash pass alone (--no-pipeline), the shard curve and the workloads
set -o pipefail
export PYTHONUNBUFFERED=1
bash scripts/gpu_full.sh || exit $?
mkdir -p gpurun_out/curve gpurun_out/wl
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/wl/cfg3_20steps.json 2>> gpurun_out/wl/err || exit 1
timeout -k 10 120 python bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu > gpurun_out/wl/cfg3_nopipe.json 2>> gpurun_out/wl/err || exit 1
for f in cfg3_20steps cfg3_nopipe; do python3 -c "import json; d=json.load(open('gpurun_out/wl/$f.json')); print('$f', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"; done
for I in 2048 4096 8192; do
  timeout -k 10 120 python bench.py --instances $I --steps 20 --warmup 3 --no-cpu > gpurun_out/curve/cfg3_${I}_d3.json 2>> gpurun_out/curve/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/curve/cfg3_${I}_d3.json')); print('curve', $I, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
done
for W in "cfg3 --seed-order le" drop64 cfg2 "cfg4 --n 256" "cfg4 --n 128"; do
  T=$(echo $W | tr -d ' -')
  timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 2 --no-cpu > gpurun_out/wl/$T.json 2>> gpurun_out/wl/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/wl/$T.json')); print('$T', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms/step')"
done
timeout -k 10 300 python bench.py --workload cfg5 --steps 2 --warmup 1 --no-cpu > gpurun_out/wl/cfg5.json 2>> gpurun_out/wl/err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/wl/cfg5.json')); print('cfg5', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms/step')"
