#!/bin/bash
# A/B of library builds on any bench workload (through gpurun), two repetitions each.
# usage: VARS="prod var_x ..." WL="drop64|cfg2|cfg3 --seed-order le|..." [STEPS=5] [TAG=x] scripts/gpu_abw.sh
# (prod = consensus-rs_amd/build/libbftsim.so, var_x = consensus-rs_amd/build/var_x/libbftsim.so)
set -o pipefail
O=gpurun_out/abw${TAG}; mkdir -p $O
export PYTHONUNBUFFERED=1
n=$(echo $WL | tr ' ' '_' | tr -d '-')
for i in 1 2; do
  for v in $VARS; do
    lib=consensus-rs_amd/build/libbftsim.so; [ $v = prod ] || lib=consensus-rs_amd/build/$v/libbftsim.so
    BFTSIM_TESTING=1 BFTSIM_LIB=$lib timeout -k 10 200 python bench.py --workload $WL --no-cpu --steps ${STEPS:-5} --warmup ${WARMUP:-1} > $O/${n}_$v.$i.json 2> $O/${n}_$v.$i.err || { tail -5 $O/${n}_$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$v.$i.json')); print('$WL', '$v', '%.3e'%d['value'], d['roofline']['kernel_ms'])"
  done
done
