#!/bin/bash
# round 3: suffix-kernel placement (prod: launch stream; var_sfx1: hash stream; var_sfx2: a thread per
# instance on the hash stream) on cfg3, and the product's small shards (chain priority below 6,144)
set -o pipefail
export PYTHONUNBUFFERED=1
TAG=_sfx VARS="prod var_sfx1 var_sfx2" WL=cfg3 STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_sfx VARS="prod var_sfx2" WL="cfg3 --instances 2048" STEPS=20 bash scripts/gpu_abw.sh || exit 1
TAG=_sfx VARS="prod var_sfx2" WL="cfg3 --instances 4096" STEPS=20 bash scripts/gpu_abw.sh || exit 1
