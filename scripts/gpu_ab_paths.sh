#!/bin/bash
# A/B of library builds on the cfg3 bench (through gpurun): scripts/gpu_ab_paths.sh name=path/to/libbftsim.so ...
# each build is benched twice, interleaved (A B C A B C), so drift of the box shows up in both
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
EXTRA=${AB_ARGS:-}
for i in 1 2; do
  for kv in "$@"; do
    name=${kv%%=*}; f=${kv#*=}
    BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu $EXTRA > gpurun_out/ab/$name.$i.json 2>> gpurun_out/ab/ab.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab/$name.$i.json')); r=d['roofline']['kernel_ms']; print('$name', round(d['value']/1e6,1), 'M/s  consensus', round(r['bft_consensus_kernel'],3), 'ms  hash', round(r['bft_hash_kernel'],3), 'ms')"
  done
done
