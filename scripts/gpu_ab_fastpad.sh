#!/bin/bash
# A/B of the FAST kernel's residency on the cfg3 bench (through gpurun): extra dynamic LDS per FAST wave
# (BFTSIM_FAST_LDS_PAD, testing only) leaves registers for chain waves beside it. Interleaved arms.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ab_fastpad
for i in 1 2; do
  for pad in 0 6000 12000 20000; do
    BFTSIM_TESTING=1 BFTSIM_FAST_LDS_PAD=$pad timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu $AB_ARGS > gpurun_out/ab_fastpad/p$pad.$i.json 2>> gpurun_out/ab_fastpad/ab.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_fastpad/p$pad.$i.json')); r=d['roofline']['kernel_ms']; print('pad $pad', round(d['value']/1e6,1), 'M/s', round(r['bft_consensus_kernel'],3), round(r['bft_hash_kernel'],3))"
  done
done
