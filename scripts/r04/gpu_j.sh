#!/bin/bash
# Global-qualified tree engine / generic / varlen accesses: the GPU suite, then the tree
# engine's nested shapes at 2M records and the Mixed / Nested benches (v9 default), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_nested_shapes.py 2097152 > $O/nested_shapes_2M.log 2>&1
rc=$?; tail -12 $O/nested_shapes_2M.log; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/b_${cfg}.json 2> $O/b_${cfg}.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('$O/b_${cfg}.json')); print('$cfg', d['value'], d['kernels_ms'])"
done
for k2 in 1 0 1; do
  for cfg in mixed40 nested; do
    FORY_ROWFMT_DECK2=$k2 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/k2_${cfg}_$k2.json 2> $O/k2_${cfg}_$k2.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json,sys; d=json.load(open('$O/k2_${cfg}_$k2.json')); print('$cfg deck2=$k2', d['value'], d['kernels_ms'])"
  done
done
