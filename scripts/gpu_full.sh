#!/bin/bash
# Round-end style GPU pass (through gpurun): every -m gpu test, smoke(), then the measurement pass
# of scripts/gpu_profile.sh. Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash scripts/gpu_profile.sh
