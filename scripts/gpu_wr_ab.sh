set -o pipefail
bash scripts/gpu_ab.sh "$@" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in "$@"; do
BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/libbftsim_$w.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/wr_$w -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2>&1 || exit $?
python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('gpurun_out/wr_$w/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if 'fast_kernel' in r['Kernel_Name']]
print('$w WRITE_SIZE MB per launch', sum(v)/len(v)*1024/1e6)"
done
