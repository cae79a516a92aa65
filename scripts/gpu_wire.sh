#!/bin/bash
# wire-codec measurement pass (through gpurun): parity tests, bench line, rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out/wireprof
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 240 --timeout-method thread > gpurun_out/wire_tests.log 2>&1 || { tail -30 gpurun_out/wire_tests.log; exit 1; }
tail -2 gpurun_out/wire_tests.log
timeout -k 10 200 python bench.py --workload wire --steps 10 --warmup 2 > gpurun_out/bench_wire.json && cat gpurun_out/bench_wire.json && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wireprof -o run --output-format csv -- python3 bench.py --workload wire --steps 10 --warmup 2 --no-cpu > gpurun_out/wireprof/bench.json 2> gpurun_out/wireprof/err.txt
rc=$?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/wireprof/run_kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PY
exit $rc
