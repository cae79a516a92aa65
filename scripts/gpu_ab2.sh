#!/bin/bash
# A/B of library builds x bench arguments on cfg3 (through gpurun):
#   scripts/gpu_ab2.sh "<lib>|<bench args>" ...   (lib: prod or a build/<lib>/libbftsim.so directory name)
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  lib=${spec%%|*}; args=${spec#*|}
  f=consensus-rs_amd/build/libbftsim.so
  [ "$lib" != "prod" ] && f=consensus-rs_amd/build/$lib/libbftsim.so
  tag=$(echo "$lib$args" | tr -c 'A-Za-z0-9' '_')
  for i in 1 2; do
    BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu $args > gpurun_out/ab/$tag.$i.json 2>> gpurun_out/ab/ab.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab/$tag.$i.json')); r=d['roofline']['kernel_ms']; print('$lib $args', round(d['value']/1e6,1), 'M/s  consensus', round(r['bft_consensus_kernel'],3), 'ms  hash', round(r['bft_hash_kernel'],3), 'ms')"
  done
done
