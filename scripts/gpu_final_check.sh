#!/bin/bash
# Final check of the committed tree (through gpurun): the whole -m gpu suite, smoke(), the default bench line and
# the sig / crypto bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit 1
for w in sig crypto; do timeout -k 10 300 python bench.py --workload $w --no-cpu > $O/$w.json 2> $O/$w.err || exit 1; done
for w in default sig crypto; do python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', '%.4g' % d['value'], d['unit'])"; done
