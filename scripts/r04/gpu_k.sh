#!/bin/bash
# Decode pass 1 straight from global for flat plans: varlen / frame parity, then the Mixed /
# Nested benches with the per-kernel times (rocprofv3 kernel trace), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04k
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/b_${cfg}.json 2> $O/b_${cfg}.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('$O/b_${cfg}.json')); print('$cfg', d['value'], d['kernels_ms'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mixed -o run -- python bench.py --config mixed40 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_mixed.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
find $O/prof_mixed -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
