#!/bin/bash
# Encode v9 without the inline per-record path (nullability-templated): varlen parity, then
# A/B v9 / v7 / round 3 on Mixed and Nested, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "varlen or mixed or collection or unaligned" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for enc in 9 7 1; do
  for cfg in mixed40 nested; do
    FORY_ROWFMT_VARENC=$enc FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_${cfg}_e${enc}.json 2> $O/ab_${cfg}_e${enc}.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json,sys; d=json.load(open('$O/ab_${cfg}_e${enc}.json')); print('$cfg enc$enc', d['value'], d['kernels_ms'])"
  done
done
grep -h "encode" $O/ab_*.err | sort | uniq -c
