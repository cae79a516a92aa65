#!/bin/bash
# Round-4 closing pass (one gpurun call): the whole -m gpu suite and smoke(), then per workload the
# measurement pass of scripts/gpu_profile.sh (bench line with the CPU baseline, rocprofv3 kernel stats,
# FETCH / WRITE / SQ PMC passes) for cfg3 (the headline, the driver's 20 steps after 5 warmup), cfg3 with
# little-endian seeds, drop64, cfg4 N=256 / N=128 and cfg2; bench lines for cfg5, crypto, sig, wire, msgpath.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
STEPS=20 WARMUP=5 NAME=r04f/cfg3 bash scripts/gpu_profile.sh cfg3 || exit 1
STEPS=20 WARMUP=5 NAME=r04f/cfg3le bash scripts/gpu_profile.sh cfg3 --seed-order le || exit 1
STEPS=5 WARMUP=1 NAME=r04f/drop64 bash scripts/gpu_profile.sh drop64 || exit 1
STEPS=5 WARMUP=1 NAME=r04f/cfg4_n256 bash scripts/gpu_profile.sh cfg4 --n 256 || exit 1
STEPS=5 WARMUP=1 NAME=r04f/cfg4_n128 bash scripts/gpu_profile.sh cfg4 --n 128 || exit 1
STEPS=10 WARMUP=2 NAME=r04f/cfg2 bash scripts/gpu_profile.sh cfg2 || exit 1
for w in cfg5 crypto sig wire msgpath; do
  timeout -k 10 600 python bench.py --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['metric'][:40], '%.4g' % d['value'], d['unit'])"
done
