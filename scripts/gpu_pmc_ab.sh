#!/bin/bash
# SQ counter passes of the cfg3 bench for library builds (through gpurun): scripts/gpu_pmc_ab.sh <suffix>...
set -o pipefail
mkdir -p gpurun_out/pmcab
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH"
for lib in "$@"; do
  f=consensus-rs_amd/build/libbftsim_$lib.so
  for k in 1 2; do
    eval P=\$P$k
    BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmcab/$lib.$k -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pipeline > gpurun_out/pmcab/$lib.$k.json 2> gpurun_out/pmcab/$lib.$k.err || exit $?
  done
  python3 - "$lib" <<'PY'
import csv, glob, sys
from collections import defaultdict
lib = sys.argv[1]
acc = defaultdict(list)
for k in (1, 2):
    for f in glob.glob(f"gpurun_out/pmcab/{lib}.{k}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "fast_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = 16384 * 100
print(lib, " ".join(f"{k}={sum(v)/len(v)/w:.1f}" for k, v in sorted(acc.items())))
PY
done
