#!/bin/bash
# Round 6, call Y: the guard allocator with every new mapping filled first, 0x00 then 0xff
# (FORY_GUARD_FILL): does the nested file's result depend on the bytes of fresh memory?
# Usage: gpu_y.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06y}
mkdir -p $O
export FORY_TEST_GUARD_ALLOC=1
for fill in 0x00 0xff; do
  FORY_GUARD_FILL=$fill timeout -k 10 300 python -u -m pytest tests/test_gpu_nested.py -m gpu -q --maxfail 10 \
    --timeout 120 --timeout-method thread > $O/pytest_fill_$fill.log 2>&1
  rc=$?
  echo "fill $fill: exit $rc"; grep -E "^FAILED|passed|failed" $O/pytest_fill_$fill.log | tail -12
  grep -q -i "illegal\|aborted\|core dumped" $O/pytest_fill_$fill.log && { echo "fault: stop"; exit 1; }
  [ $rc -le 1 ] || exit 1
done
exit 0
