#!/bin/bash
# r04sig: the secp256k1 product with the carry-add addend (product) vs the round-3 form (build/var_sig0):
# GPU sig and crypto tests, then sig / crypto bench lines for both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04sig; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sig or crypto or msgpath or ledger" > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
for v in prod sig0; do
  if [ $v = prod ]; then L=consensus-rs_amd/build/libbftsig.so; else L=consensus-rs_amd/build/var_$v/libbftsig.so; fi
  for w in sig crypto; do
    env BFTSIM_TESTING=1 BFTSIG_LIB=$L timeout -k 10 600 python bench.py --workload $w --no-cpu > $O/${w}_$v.json 2> $O/${w}_$v.err || exit 1
    python3 -c "import json; d=json.load(open('$O/${w}_$v.json')); r=d.get('roofline') or {}; print('${w}_$v', '%.4g' % d['value'], d['unit'], r.get('frac'))"
  done
done
