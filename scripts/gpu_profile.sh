#!/bin/bash
# Measurement pass of one workload (through gpurun): bench line with the CPU baseline, rocprofv3 kernel
# stats, and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, and WRITE_SIZE again with an L2 eviction after every
# kernel of unpipelined launches for per-kernel write attribution) — counters never share a pass with
# traces other than --kernel-trace/--stats. Summary: <out>/pmc_summary.json (scripts/pmc_summary.py).
# usage: [NAME=dir] scripts/gpu_profile.sh [workload] [extra bench args...]   (outputs under gpurun_out/prof/<NAME or workload>)
set -o pipefail
W=${1:-cfg3}; shift
X="$*"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/prof/${NAME:-$W}
mkdir -p $R
S=${STEPS:-10}; PS=${PSTEPS:-3}; WU=${WARMUP:-2}; PWU=${PWARMUP:-1}
lscpu | grep -E "Model name|^CPU\(s\)" > $R/host_cpu.txt; nproc > $R/host_nproc.txt
timeout -k 10 600 python bench.py --workload $W $X --steps $S --warmup $WU > $R/bench.json 2> $R/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/stats -o run --output-format csv -- python3 bench.py --workload $W $X --steps $S --warmup $WU --no-cpu > $R/stats.json 2> $R/stats.err && \
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/fetch -o run --output-format csv -- python3 bench.py --workload $W $X --steps $PS --warmup $PWU --no-cpu > $R/fetch.json 2> $R/fetch.err && \
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/write -o run --output-format csv -- python3 bench.py --workload $W $X --steps $PS --warmup $PWU --no-cpu > $R/write.json 2> $R/write.err && \
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $R/sq -o run --output-format csv -- python3 bench.py --workload $W $X --steps $PS --warmup $PWU --no-cpu > $R/sq.json 2> $R/sq.err && \
BFTSIM_TESTING=1 BFTSIM_PMC_EVICT=1 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/write_evict -o run --output-format csv -- python3 bench.py --workload $W $X --steps $PS --warmup $PWU --no-cpu --no-pipeline > $R/write_evict.json 2> $R/write_evict.err && \
python3 scripts/pmc_summary.py $R $R/pmc_summary.json > /dev/null
rc=$?
echo "$W rc=$rc"
python3 -c "import json; d=json.load(open('$R/bench.json')); print(d['config']['workload'], round(d['value']/1e6,2), 'M/s', d['roofline']['kernel_ms'], 'cpu', d.get('cpu_baseline',{}).get('value'))" 2>/dev/null
exit $rc
