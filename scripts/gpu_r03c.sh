#!/bin/bash
# round 3: SEEDED FAST (little-endian seeds) parity + A/B of its occupancy; general-kernel section stamps
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q -k "le or little" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in prod var_w4s; do
    lib=consensus-rs_amd/build/libbftsim.so; [ $v = prod ] || lib=consensus-rs_amd/build/$v/libbftsim.so
    BFTSIM_TESTING=1 BFTSIM_LIB=$lib timeout -k 10 120 python bench.py --seed-order le --no-cpu --steps 10 --warmup 2 > $O/le_$v.$i.json 2> $O/le_$v.$i.err || { tail -5 $O/le_$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/le_$v.$i.json')); print('$v', '%.3e'%d['value'], d['roofline']['kernel_ms'])"
  done
done
bash scripts/gpu_stamps_general.sh > /dev/null 2>&1; rc=$?; cp gpurun_out/stamps_general.txt $O/ 2>/dev/null; cat $O/stamps_general.txt; exit $rc
