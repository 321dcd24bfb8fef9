#!/bin/bash
# XCD-run tile order (FORY_ROWFMT_VARXCD) A/B on the varlen tile kernels: Mixed and Nested,
# encode v7 / round 3 / v8, decode; one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mixed or nested or varlen" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for xcd in 0 -1 16 4; do
  for enc in 7 1 0; do
    for cfg in mixed40 nested; do
      FORY_ROWFMT_VARXCD=$xcd FORY_ROWFMT_VARENC=$enc timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_${cfg}_x${xcd}_e${enc}.json 2> $O/ab_${cfg}_x${xcd}_e${enc}.err
      rc=$?; [ $rc -eq 0 ] || exit $rc
      python -c "import json,sys; d=json.load(open('$O/ab_${cfg}_x${xcd}_e${enc}.json')); print('$cfg xcd$xcd enc$enc', d['value'], d['kernels_ms'])"
    done
  done
done
