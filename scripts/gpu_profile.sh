#!/bin/bash
# Full measurement pass (through gpurun): bench with the CPU baseline, rocprofv3 kernel stats,
# and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) — counters never share a pass with traces
# other than --kernel-trace/--stats. Summary: gpurun_out/prof/pmc_summary.json (scripts/pmc_summary.py).
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/prof
nproc > gpurun_out/host_nproc.txt; lscpu | grep -E "Model name|^CPU\(s\)" > gpurun_out/host_cpu.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample ${CPU_SAMPLE:-16384} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/stats -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $R/stats.json 2> $R/stats.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $R/fetch.json 2> $R/fetch.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $R/write.json 2> $R/write.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $R/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $R/sq.json 2> $R/sq.err && \
python3 scripts/pmc_summary.py $R $R/pmc_summary.json > /dev/null
rc=$?
echo "rc=$rc"
cat gpurun_out/bench.json
find $R -name "*kernel_stats.csv" | head -3
exit $rc
