#!/bin/bash
# wave-count tail probe: one workload at several instance counts (no CPU leg)
set -o pipefail
O=gpurun_out/tail; mkdir -p $O
for n in $NS; do
  timeout -k 10 200 python bench.py --workload $WL --instances $n --no-cpu --steps 5 --warmup 1 > $O/${WL}_$n.json 2> $O/${WL}_$n.err || { tail -5 $O/${WL}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${WL}_$n.json')); print('$WL', $n, '%.3e'%d['value'], d['roofline']['kernel_ms'])"
done
