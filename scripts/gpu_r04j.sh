#!/bin/bash
# round 4: canonical tick checks in integer form + plain LDS histogram; defaults (batch/depth) A/B at 16k; SQ PMC
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $BARGS > $O/$name.json 2>> $O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
BARGS="" run cfg3
BARGS="--no-pipeline" run cfg3_nopipe
for r in 1 2; do
  for B in 2 3 4; do for D in 6 8; do BARGS="--hash-batch $B --pipeline-depth $D" run c16k_b${B}_d${D}_r$r; done; done
done
for I in 2048 4096 8192; do BARGS="--instances $I" run c$I; done
BARGS="--seed-order le --steps 10" run cfg3_le
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/sq -o run --output-format csv -- python3 bench.py --no-pipeline --steps 5 --warmup 2 --no-cpu > $O/sq.json 2> $O/sq.err || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r04j/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "consensus_fast" in k or "chain" in k:
        print(k, {c: "%.3g" % v for c, v in d.items()})
PY
