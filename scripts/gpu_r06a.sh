set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > $O/pipe.log 2>&1; rc=$?
tail -25 $O/pipe.log; [ $rc -eq 0 ] || exit $rc
for a in on off; do
  if [ $a = off ]; then export BFTSIM_TESTING=1 BFTSIM_HASH_SPEC=0; fi
  timeout -k 10 200 python bench.py --no-cpu > $O/cfg3_$a.json 2> $O/cfg3_$a.err || { tail -5 $O/cfg3_$a.err; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu --instances 2048 > $O/s2048_$a.json 2> $O/s2048_$a.err || { tail -5 $O/s2048_$a.err; exit 1; }
  python3 -c "import json
for f in ('cfg3','s2048'):
  d=json.load(open('$O/'+f+'_$a.json')); print(f, '$a', '%.4g' % d['value'], d['ms_per_step'])"
done
