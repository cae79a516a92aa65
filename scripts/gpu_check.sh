#!/bin/bash
# One GPU check of the working tree (through gpurun): the whole -m gpu suite, then the default bench line, then
# optional extra steps named in $EXTRA (each a command line run from the repo root, all under their own
# time limits inside the called scripts). Stops at the first failure.
# usage: OUT=<name> EXTRA="cmd1;cmd2" bash scripts/gpu_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-check}; mkdir -p $O
if [ -z "$NOSUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${SUITE_ARGS} > $O/gpu_suite.log 2>&1; rc=$?
  tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/default.json')); print('default', '%.4g' % d['value'], d['unit'], d['roofline']['kernel_ms'])"
fi
IFS=';' read -ra STEPS_ <<< "$EXTRA"
for c in "${STEPS_[@]}"; do
  [ -z "$c" ] && continue
  echo "== $c"
  bash -c "$c" || exit 1
done
