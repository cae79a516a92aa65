set -o pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONUNBUFFERED=1
AB_ARGS="--workload cfg5 --steps 1 --warmup 1" bash scripts/gpu_ab_paths.sh new=consensus-rs_amd/build/libbftsim.so o3=consensus-rs_amd/build/var_o3/libbftsim.so o3ip=consensus-rs_amd/build/var_o3ip/libbftsim.so && \
AB_ARGS="--workload cfg2" bash scripts/gpu_ab_paths.sh c2new=consensus-rs_amd/build/libbftsim.so c2w4=consensus-rs_amd/build/var_w4/libbftsim.so
