#!/bin/bash
# Round 6, call X: guard-page allocator (tests/guard_alloc/): every torch tensor ends at an
# unmapped granule, so a kernel reading past a tensor's end faults at once, in the test
# that does it. First the tree-engine and varlen files, then (if clean) frames and windows.
# Usage: gpu_x.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06x}
mkdir -p $O
export FORY_TEST_GUARD_ALLOC=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_treecol.py tests/test_gpu_v9.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_guard_a.log 2>&1
rc=$?
echo "(a) nested, treecol, v9: exit $rc"; tail -40 $O/pytest_guard_a.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_windows.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_guard_b.log 2>&1
rc=$?
echo "(b) frames, windows: exit $rc"; tail -40 $O/pytest_guard_b.log
exit $rc
