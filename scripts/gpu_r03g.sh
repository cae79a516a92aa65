#!/bin/bash
# round 3: secp256k1 recover variants, then the S < 64 summary change (product vs var_head) on cfg2 / cfg5
set -o pipefail
export PYTHONUNBUFFERED=1
VARS="var_sig_old var_sig_w1 var_sig_w2" bash scripts/gpu_ab_sig.sh || exit 1
TAG=_g VARS="var_head prod" WL=cfg2 bash scripts/gpu_abw.sh || exit 1
TAG=_g VARS="var_head prod" WL="cfg5 --instances 32768 --heights 2000" STEPS=2 bash scripts/gpu_abw.sh || exit 1
