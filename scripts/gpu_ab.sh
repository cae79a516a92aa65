#!/bin/bash
# A/B of library builds on the cfg3 bench (through gpurun): scripts/gpu_ab.sh <suffix>... ("" = product)
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for lib in "$@"; do
  f=consensus-rs_amd/build/libbftsim${lib:+_$lib}.so
  [ "$lib" = "prod" ] && f=consensus-rs_amd/build/libbftsim.so
  for i in 1 2; do
    BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab/$lib.$i.json 2>> gpurun_out/ab/ab.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab/$lib.$i.json')); r=d['roofline']['kernel_ms']; print('$lib', round(d['value']/1e6,1), 'M/s  consensus', round(r['bft_consensus_kernel'],3), 'ms  hash', round(r['bft_hash_kernel'],3), 'ms')"
  done
done
