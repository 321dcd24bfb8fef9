#!/bin/bash
# Branch-free loads in the nested layout walk (round-3 encode) and the decode's tile-start
# offsets behind the DMA: varlen / frame parity, then Mixed / Nested benches twice, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_nested.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in mixed40 nested; do
    timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/b_${cfg}_$rep.json 2> $O/b_${cfg}_$rep.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json,sys; d=json.load(open('$O/b_${cfg}_$rep.json')); print('$cfg', d['value'], d['kernels_ms'])"
  done
done
