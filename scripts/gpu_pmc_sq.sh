#!/bin/bash
# SQ instruction counters of the cfg3 bench for library builds (through gpurun):
#   scripts/gpu_pmc_sq.sh name=path/to/libbftsim.so ...   -> gpurun_out/pmcsq/<name>/ + one summary line each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=${SQ_COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY"}
for kv in "$@"; do
  name=${kv%%=*}; f=${kv#*=}
  R=gpurun_out/pmcsq/$name; mkdir -p $R
  BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $R -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $R/b.json 2> $R/b.err || exit $?
  python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
f = glob.glob(f"{R}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "fast_kernel" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = {k: acc[k] / n[k] for k in acc}
views = 1638400.0
print(R.split("/")[-1], " ".join(f"{k.replace('SQ_','')}={d[k]/views:.1f}" for k in sorted(d) if k not in ("SQ_WAVES",)), "(per instance-round)")
PY
done
