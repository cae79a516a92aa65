#!/bin/bash
# A/B of general-kernel builds on cfg4 N=256 (and parity of the variant on the N > 64 cases)
# usage: VARS="var_a var_b" scripts/gpu_ab_cfg4.sh   (consensus-rs_amd/build/<var>/libbftsim.so)
set -o pipefail
O=gpurun_out/ab_cfg4${TAG}; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in $VARS; do
  BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/$v/libbftsim.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "256 or 128 or 200 or 100 or 65" --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
  tail -1 $O/parity_$v.log
done
for i in 1 2; do
  for v in prod $VARS; do
    env=""; [ $v = prod ] || env="BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/$v/libbftsim.so"
    env $env timeout -k 10 200 python bench.py --workload cfg4 --n ${NV:-256} ${XARGS} --no-cpu --steps 3 --warmup 1 > $O/$v.$i.json 2> $O/$v.$i.err || { tail -5 $O/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$i.json')); print('$v', '%.3e'%d['value'], d['roofline']['kernel_ms'])"
  done
done
