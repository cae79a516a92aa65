# round 6 A/B driver (through gpurun): ARMS="step;step;..." with steps
#   tests <pytest args>              GPU tests, stop at the first failure
#   run <name> [VAR=v ...] -- <bench args>     one bench line into $O/<name>.json
#   trace <name> [VAR=v ...] -- <bench args>   the same under rocprofv3 --kernel-trace: timeline + overlap summaries
#   pmc <name> "<counters>" [VAR=v ...] -- <bench args>   one --pmc pass, each counter summed per kernel family
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06b}; mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  local ev=()
  while [ "$1" != "--" ]; do ev+=("$1"); shift; done; shift
  env "${ev[@]}" timeout -k 10 200 python bench.py --no-cpu "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', '%.4g' % d['value'], d['ms_per_step'])"
}
trace() {  # name, env..., -- bench args
  local name=$1; shift
  local ev=()
  while [ "$1" != "--" ]; do ev+=("$1"); shift; done; shift
  mkdir -p $O/tr_$name
  env "${ev[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$name -o tr -- python3 bench.py --no-cpu "$@" > $O/tr_$name.json 2>$O/tr_$name.err || { tail -5 $O/tr_$name.err; exit 1; }
  f=$(find $O/tr_$name -name '*kernel_trace.csv' | head -1)
  python3 scripts/trace_timeline.py $f --last 20 > $O/timeline_$name.txt
  python3 scripts/trace_overlap.py $f --last 20 > $O/overlap_$name.txt
  rm -f $f
}
apitrace() {  # name, env..., -- bench args: HIP API call statistics (rocprofv3 --hip-trace --stats)
  local name=$1; shift
  local ev=()
  while [ "$1" != "--" ]; do ev+=("$1"); shift; done; shift
  mkdir -p $O/api_$name
  env "${ev[@]}" timeout -k 10 200 rocprofv3 --hip-trace --stats --output-format csv -d $O/api_$name -o api -- python3 bench.py --no-cpu "$@" > $O/api_$name.json 2>$O/api_$name.err || { tail -5 $O/api_$name.err; exit 1; }
  find $O/api_$name -name '*hip_api_stats.csv' -exec cp {} $O/api_stats_$name.csv \;
  find $O/api_$name -name '*.csv' -size +2M -delete
}
pmc() {  # name "counters" env..., -- bench args: one rocprofv3 --pmc pass, counters summed per kernel
  local name=$1 ctr=$2; shift 2
  local ev=()
  while [ "$1" != "--" ]; do ev+=("$1"); shift; done; shift
  mkdir -p $O/pmc_$name
  env "${ev[@]}" timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$name -o pmc -- python3 bench.py --no-cpu "$@" > $O/pmc_$name.json 2>$O/pmc_$name.err || { tail -5 $O/pmc_$name.err; exit 1; }
  f=$(find $O/pmc_$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_by_kernel.py $f > $O/pmc_$name.txt && cat $O/pmc_$name.txt
  find $O/pmc_$name -name '*.csv' -size +2M -delete
}
tests() {  # pytest files...: the GPU tests named, stop at the first failure
  timeout -k 10 800 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
}
IFS=';' read -ra STEPS_ <<< "$ARMS"
for c in "${STEPS_[@]}"; do
  [ -z "$c" ] && continue
  eval "$c" || exit 1
done
