#!/bin/bash
# Encode v7: varlen parity first (every engine), then the full suite, smoke, bench with
# the C2/C3 extra lines, and an A/B of the v7 vs round-3 encode on the Mixed/Nested benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for enc in 0 1; do
    for cfg in mixed40 nested; do
      FORY_ROWFMT_VARENC=$enc FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_${cfg}_enc${enc}_$rep.json 2> $O/ab_${cfg}_enc${enc}_$rep.err
      rc=$?; [ $rc -eq 0 ] || exit $rc
      python -c "import json,sys; d=json.load(open('$O/ab_${cfg}_enc${enc}_$rep.json')); print('$cfg enc$enc rep$rep', d['value'], d['kernels_ms'])"
    done
  done
done
