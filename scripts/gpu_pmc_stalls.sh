#!/bin/bash
# Stall counters of one bench command (through gpurun): SQ wait / issue / instruction-fetch counters in one pass,
# the instruction cache's hits and misses in a second (counters never share a pass with traces).
# usage: NAME=<dir> bash scripts/gpu_pmc_stalls.sh <bench args...>     (outputs under gpurun_out/stalls/<NAME>)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/stalls/${NAME:-run}; mkdir -p $R
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VALU -d $R/sq -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $R/sq.json 2> $R/sq.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $R/sqc -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $R/sqc.json 2> $R/sqc.err
rc=$?
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(R + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bft_" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k, {c: "%.4g" % x for c, x in sorted(v.items())})
PY
exit $rc
