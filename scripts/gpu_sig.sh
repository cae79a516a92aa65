#!/bin/bash
# secp256k1 measurement pass (through gpurun): parity tests, the multiply-add peak, throughput, and a
# rocprofv3 kernel trace of the throughput run (summary in gpurun_out/sigprof).
set -o pipefail
mkdir -p gpurun_out/sigprof
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sig.py -x -q --timeout 240 --timeout-method thread > gpurun_out/sig_tests.log 2>&1 || { tail -30 gpurun_out/sig_tests.log; exit 1; }
tail -2 gpurun_out/sig_tests.log
timeout -k 10 60 consensus-rs_amd/build/mad_peak > gpurun_out/mad_peak.json && cat gpurun_out/mad_peak.json && \
timeout -k 10 200 python scripts/sig_bench.py --n 262144 --reps 3 > gpurun_out/sig_bench.json && cat gpurun_out/sig_bench.json && \
timeout -k 10 200 python bench.py --workload sig --steps 10 --warmup 2 > gpurun_out/bench_sig.json && cat gpurun_out/bench_sig.json && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sigprof -o run --output-format csv -- python3 bench.py --workload sig --steps 10 --warmup 2 --no-cpu > gpurun_out/sigprof/bench.json 2> gpurun_out/sigprof/err.txt
rc=$?
cat gpurun_out/sigprof/run_kernel_stats.csv 2>/dev/null | cut -c1-150
exit $rc
