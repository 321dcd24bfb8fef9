#!/bin/bash
# Encode v8 (16-B column loads): varlen parity, then A/B v8 / v7 (VARENC=7) / round 3 (VARENC=1), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for enc in 0 7 1; do
    for cfg in mixed40; do
      FORY_ROWFMT_VARENC=$enc FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_${cfg}_enc${enc}_$rep.json 2> $O/ab_${cfg}_enc${enc}_$rep.err
      rc=$?; [ $rc -eq 0 ] || exit $rc
      python -c "import json,sys; d=json.load(open('$O/ab_${cfg}_enc${enc}_$rep.json')); print('$cfg enc$enc rep$rep', d['value'], d['kernels_ms'])"
    done
  done
done
grep -h "encode" $O/ab_*_1.err | sort | uniq -c
