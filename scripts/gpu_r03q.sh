#!/bin/bash
# round 3: small shards in steady state (20 steps after 5 warmup launches, the driver's setting):
# chains at priority 3 below 6,144 instances (prod) vs never (var_noprio)
set -o pipefail
export PYTHONUNBUFFERED=1
for I in 2048 4096; do
  TAG=_q WARMUP=5 VARS="prod var_noprio" WL="cfg3 --instances $I" STEPS=20 bash scripts/gpu_abw.sh || exit 1
done
