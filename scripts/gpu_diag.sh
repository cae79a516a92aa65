#!/bin/bash
# diagnostics (through gpurun): A/B of the product library against a baseline build, the counter
# list, and a PC-sampling pass of the cfg3 bench
set -o pipefail
mkdir -p gpurun_out/diag
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/diag
for lib in base ""; do
  f=consensus-rs_amd/build/libbftsim${lib:+_$lib}.so
  for i in 1 2; do
    BFTSIM_TESTING=1 BFTSIM_LIB=$f timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > $D/ab_${lib:-new}_$i.json 2>> $D/ab.err || exit $?
    python -c "import json,sys; d=json.load(open('$D/ab_${lib:-new}_$i.json')); print('$f', round(d['value']/1e6,1), 'M/s', round(d['roofline']['kernel_ms']['bft_consensus_kernel'],3), 'ms')"
  done
done
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10 -d $D/pcs -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $D/pcs.json 2> $D/pcs.err
echo "pcs rc=$?"; tail -5 $D/pcs.err; find $D/pcs -type f | head; 
exit 0
