#!/bin/bash
# r04p: drop draws with hoisted products (philox_drop) — parity suite (drops, crashes, resume), Philox rate,
# drop64 A/B: resume kernel at 3 waves/SIMD (product, 276 B/lane scratch) vs 2 (build/var_r2, no scratch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=8
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 60 ./tools/philox_rate > $O/philox_rate.txt 2>&1 && cat $O/philox_rate.txt && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or pipeline or fullsize" > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
for v in prod var_r2; do
  if [ $v = prod ]; then L=consensus-rs_amd/build/libbftsim.so; else L=consensus-rs_amd/build/$v/libbftsim.so; fi
  BFTSIM_TESTING=1 BFTSIM_LIB=$L timeout -k 10 300 python bench.py --workload drop64 --steps 5 --warmup 1 --no-cpu > $O/drop64_$v.json 2> $O/drop64_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/drop64_$v.json')); print('$v', round(d['value']/1e6,2), 'M/s', d['ms_per_step'])"
done
