#!/bin/bash
# round 3: gpu_r03m.sh (v_perm prefix: parity + A/B) then gpu_r03n.sh (chain priority, kernel stats)
set -o pipefail
bash scripts/gpu_r03m.sh || exit 1
bash scripts/gpu_r03n.sh || exit 1
