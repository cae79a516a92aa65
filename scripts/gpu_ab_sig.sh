#!/bin/bash
# A/B of libbftsig builds (through gpurun): secp parity of the product build, then the sig and crypto bench
# lines of each arm, interleaved.  scripts/gpu_ab_sig.sh name=dir ...  (dir holds libbftsig.so + libbftsim.so;
# "prod" = consensus-rs_amd/build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/ab_sig; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sig.py tests/test_gpu_crypto.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for arm in "$@"; do
  name=${arm%%=*}; d=${arm#*=}
  BFTSIM_TESTING=1 BFTSIG_LIB=$d/libbftsig.so BFTSIM_LIB=$d/libbftsim.so timeout -k 10 300 python bench.py --workload sig --no-cpu > $O/sig_${name}_$rep.json 2> $O/sig_${name}_$rep.err || exit 1
  BFTSIM_TESTING=1 BFTSIG_LIB=$d/libbftsig.so BFTSIM_LIB=$d/libbftsim.so timeout -k 10 300 python bench.py --workload crypto --no-cpu > $O/crypto_${name}_$rep.json 2> $O/crypto_${name}_$rep.err || exit 1
  python3 -c "
import json
for w in ('sig','crypto'):
    d=json.load(open('$O/'+w+'_${name}_$rep.json')); print(w, '$name', '%.4g' % d['value'], d['unit'], round(d['ms_per_step'],3))"
done
done
