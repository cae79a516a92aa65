#!/bin/bash
# A/B of libbftsig builds: GPU sig parity per variant, then the sig bench (recoveries/s) twice each
# usage: VARS="var_a var_b" scripts/gpu_ab_sig.sh   (consensus-rs_amd/build/<var>/libbftsig.so; prod = build/libbftsig.so)
set -o pipefail
O=gpurun_out/ab_sig; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in $VARS; do
  lib=consensus-rs_amd/build/libbftsig.so; [ $v = prod ] || lib=consensus-rs_amd/build/$v/libbftsig.so
  BFTSIM_TESTING=1 BFTSIG_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_sig.py -x -q --timeout 240 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.log)"
done
for i in 1 2; do
  for v in $VARS; do
    lib=consensus-rs_amd/build/libbftsig.so; [ $v = prod ] || lib=consensus-rs_amd/build/$v/libbftsig.so
    BFTSIM_TESTING=1 BFTSIG_LIB=$lib timeout -k 10 200 python bench.py --workload sig --steps 5 --warmup 1 --no-cpu > $O/$v.$i.json 2> $O/$v.$i.err || { tail -5 $O/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$i.json')); r=d['roofline']; print('$v', '%.3e'%d['value'], 'frac', round(r['frac'],3), r.get('kernel_ms'))"
  done
done
