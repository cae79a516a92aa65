#!/bin/bash
# Round-4 closing pass after the unrolled pair Keccak: the whole -m gpu suite and smoke(), the cfg3 measurement
# pass (bench + rocprof stats + PMC, 20 steps after 5 warmup), the strong-scaling shards and LE bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/closing; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
STEPS=20 WARMUP=5 NAME=closing/cfg3 bash scripts/gpu_profile.sh cfg3 || exit 1
for I in 2048 4096 8192; do
  STEPS=20 WARMUP=5 NAME=closing/cfg3_$I bash scripts/gpu_profile.sh cfg3 --instances $I || exit 1
done
timeout -k 10 300 python bench.py --seed-order le --steps 20 --warmup 5 > $O/cfg3le.json 2> $O/cfg3le.err || exit 1
python3 -c "import json; d=json.load(open('$O/cfg3le.json')); print('le', '%.4g' % d['value'])"
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit 1
python3 -c "import json; d=json.load(open('$O/default.json')); print('default', '%.4g' % d['value'], d['steps'], d['warmup'])"
