#!/bin/bash
# r04t: the LE launch-stream sweep (gpu_r04s.sh), then per-section stamps of the general kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r04s.sh || exit 1
bash scripts/gpu_stamps_general.sh
