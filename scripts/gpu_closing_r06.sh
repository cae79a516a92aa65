#!/bin/bash
# Round-6 closing measurement passes (through gpurun), one group of workloads per call so each call stays well
# inside gpurun's limit:  bash scripts/gpu_closing_r06.sh A|B|C|D|E
#   E: the shard curve (2,048 .. 16,384 instances per GPU) of the strong-scaling workload
#   A: the whole -m gpu suite, smoke(), cfg3 (the headline, 20 steps after 5 warmup) and its 2,048-instance shard
#   B: cfg5 (one 10,000-height step), cfg2, drop64
#   C: cfg4 N = 256 and N = 128, little-endian cfg3
#   D: the bench lines of every workload again, now reading this round's PMC summaries (profiles/r06/)
# Each workload: scripts/gpu_profile.sh (bench line, rocprofv3 stats, FETCH / WRITE / SQ PMC passes and the
# L2-eviction write-attribution pass) into gpurun_out/prof/r06/<name>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/closing_r06; mkdir -p $O
case "$1" in
A)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
  tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  STEPS=20 WARMUP=5 NAME=r06 bash scripts/gpu_profile.sh cfg3 || exit 1
  STEPS=20 WARMUP=5 NAME=r06/cfg3_2048 bash scripts/gpu_profile.sh cfg3 --instances 2048 || exit 1
  ;;
B)
  STEPS=1 WARMUP=0 PSTEPS=1 PWARMUP=0 NAME=r06/cfg5 bash scripts/gpu_profile.sh cfg5 || exit 1
  NAME=r06/cfg2 bash scripts/gpu_profile.sh cfg2 || exit 1
  STEPS=5 WARMUP=1 PSTEPS=1 PWARMUP=0 NAME=r06/drop64 bash scripts/gpu_profile.sh drop64 || exit 1
  ;;
C)
  STEPS=5 WARMUP=1 PSTEPS=1 PWARMUP=0 NAME=r06/cfg4_n256 bash scripts/gpu_profile.sh cfg4 --n 256 || exit 1
  STEPS=5 WARMUP=1 PSTEPS=1 PWARMUP=0 NAME=r06/cfg4_n128 bash scripts/gpu_profile.sh cfg4 --n 128 || exit 1
  STEPS=20 WARMUP=5 NAME=r06/cfg3le bash scripts/gpu_profile.sh cfg3 --seed-order le || exit 1
  ;;
E)
  # the shard curve of the strong-scaling workload: instances per GPU 2,048 .. 16,384, twice each
  mkdir -p $O/curve
  for rep in 1 2; do for n in 2048 4096 8192 16384; do
    timeout -k 10 300 python bench.py --no-cpu --instances $n > $O/curve/n${n}_$rep.json 2> $O/curve/n${n}_$rep.err || { tail -5 $O/curve/n${n}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/curve/n${n}_$rep.json')); print('$n', '%.4g' % d['value'], d['config']['host_enqueue_ms'])"
  done; done
  ;;
D)
  mkdir -p $O/lines
  for w in "cfg3" "cfg3 --instances 2048" "cfg3 --seed-order le" "cfg5 --steps 1 --warmup 0" "cfg2" "drop64 --steps 5 --warmup 1" \
           "cfg4 --n 256 --steps 5 --warmup 1" "cfg4 --n 128 --steps 5 --warmup 1" "sig" "crypto" "wire"; do
    n=$(echo $w | tr ' ' '_' | tr -d '-')
    timeout -k 10 400 python bench.py --workload $w > $O/lines/$n.json 2> $O/lines/$n.err || { tail -5 $O/lines/$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lines/$n.json')); print('$n', '%.4g' % d['value'], d['unit'], (d.get('roofline') or {}).get('frac'))"
  done
  ;;
esac
