#!/bin/bash
# round 3: the whole GPU suite on the current build, then bench lines of the consensus workloads (no CPU leg)
set -o pipefail
O=gpurun_out/r03b${TAG}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
# WORKLOADS: '|'-separated bench argument lists
IFS='|' read -ra WLS <<< "${WORKLOADS:-cfg3|cfg3 --seed-order le|drop64|cfg4 --n 256|cfg2}"
for w in "${WLS[@]}"; do
  n=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 240 python bench.py --workload $w --no-cpu --steps 10 --warmup 2 > $O/b_$n.json 2> $O/b_$n.err || { echo "bench $w failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b_$n.json')); print('$w', '%.3e'%d['value'], d['roofline']['kernel_ms'])"
done
