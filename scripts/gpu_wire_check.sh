#!/bin/bash
# wire codec: GPU tests, A/B of the decoder (scripts/gpu_wire_ab.sh), rocprof kernel stats (through gpurun)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_wire_block.py tests/test_gpu_msgpath.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/wire_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wire_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_wire_ab.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wprof -o run --output-format csv -- python3 bench.py --workload wire --steps 5 --warmup 1 --no-cpu > gpurun_out/wprof.json 2> gpurun_out/wprof.err || exit $?
python3 - <<'PY'
import csv, glob
for r in csv.DictReader(open(glob.glob("gpurun_out/wprof/**/run_kernel_stats.csv", recursive=True)[0])):
    print(r["Name"][:50], r["AverageNs"])
PY
