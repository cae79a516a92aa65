#!/bin/bash
# round 3, first GPU pass: the new GPU tests (timed-mode parity at full size, phase-cap FAST cases),
# then short bench lines of every consensus workload on this box (no CPU leg)
set -o pipefail
mkdir -p gpurun_out/r03a
export PYTHONUNBUFFERED=1
O=gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py "tests/test_gpu_parity.py::test_gpu_matches_oracle[n64-byz21-cap3]" "tests/test_gpu_parity.py::test_gpu_matches_oracle[n64-byz21-cap4]" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in "cfg3" "cfg3 --seed-order le" "drop64" "cfg2" "cfg4 --n 256" "cfg4 --n 64" "cfg5 --steps 1 --warmup 0"; do
  n=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 240 python bench.py --workload $w --no-cpu $( [[ "$w" == cfg5* ]] || echo "--steps 10 --warmup 2") > $O/b_$n.json 2> $O/b_$n.err || { echo "bench $w failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b_$n.json')); print('$w', '%.3e'%d['value'], d['roofline']['kernel_ms'])"
done
