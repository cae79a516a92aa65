#!/bin/bash
# round 4: the canonical tick (whole steady-state tick in closed form): GPU suite, cfg3 + shard curve, rocprof stats
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="" run cfg3
BARGS="--no-pipeline" run cfg3_nopipe
for D in 3 4 6 8; do BARGS="--pipeline-depth $D" run cfg3_d$D; done
for I in 2048 4096 8192; do BARGS="--instances $I" run c$I; done
BARGS="--instances 2048 --pipeline-depth 8 --hw-queues 10" run c2048_d8_q10
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_bench.json 2> $O/prof.err || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
