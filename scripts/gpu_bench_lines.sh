#!/bin/bash
# Bench lines only (through gpurun), no CPU baseline: one `python bench.py --workload <args> --no-cpu` per
# argument, each under its own time limit, into gpurun_out/<OUT>/<name>.json; prints value and kernel ms.
# usage: OUT=<name> bash scripts/gpu_bench_lines.sh "cfg5 --steps 2 --warmup 1" "cfg3" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-lines}; mkdir -p $O
for w in "$@"; do
  n=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --workload $w --no-cpu > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', '%.4g' % d['value'], d['unit'], (d.get('roofline') or {}).get('kernel_ms'))"
done
