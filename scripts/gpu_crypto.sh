#!/bin/bash
# real-crypto mode: GPU tests, then the crypto bench line and the cfg3 line (stdout must be one JSON line)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_crypto.py tests/test_gpu_comm.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/crypto_tests.log 2>&1
rc=$?
tail -3 gpurun_out/crypto_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/crypto_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --workload crypto --steps 3 --warmup 1 > gpurun_out/bench_crypto.json 2> gpurun_out/bench_crypto.err || exit $?
cat gpurun_out/bench_crypto.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(round(d['value']/1e6,1), 'M instance-rounds/s', d['config']['stats_allreduce'])"
