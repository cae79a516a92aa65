#!/bin/bash
# round 4: resume grid hint + the canonical ticks' own loop: GPU suite, cfg3 + shards, SQ PMC of cfg3
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="" run cfg3
BARGS="" run cfg3_b
BARGS="--no-pipeline" run cfg3_nopipe
for I in 2048 4096; do BARGS="--instances $I" run c$I; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_bench.json 2> $O/prof.err || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/sq -o run --output-format csv -- python3 bench.py --no-pipeline --steps 5 --warmup 2 --no-cpu > $O/sq.json 2> $O/sq.err || exit 1
grep -E "Name|consensus|resume|chain|suffix" $O/prof/run_kernel_stats.csv | cut -c1-150
