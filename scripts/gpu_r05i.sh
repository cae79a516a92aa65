set -o pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05i
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_ledger.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05i/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--workload cfg5 --steps 1 --warmup 1" bash scripts/gpu_ab_paths.sh c5prev=consensus-rs_amd/build/var_prev/libbftsim.so c5new=consensus-rs_amd/build/libbftsim.so
