set -o pipefail
mkdir -p gpurun_out/wab
for i in 1 2; do for v in old=consensus-rs_amd/build/ab_wire_old/libbftwire.so new=consensus-rs_amd/build/libbftwire.so; do
  n=${v%%=*}; f=${v#*=}
  BFTSIM_TESTING=1 BFTWIRE_LIB=$f timeout -k 10 120 python bench.py --workload wire --steps 10 --warmup 2 --no-cpu > gpurun_out/wab/$n.$i.json 2>> gpurun_out/wab/err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/wab/$n.$i.json')); print('$n', '%.3e'%d['value'], d['roofline']['frac'])"
done; done
