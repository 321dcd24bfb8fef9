#!/bin/bash
# Round 6, call W: the workspace-fill diagnostic split in two (fury_amd/format/encoder.py,
# FORY_TEST_WS_FILL=0xff). (a) the fill before each encode and before the first
# decode_sizes only: the state decode_sizes leaves for decode is kept; (b) the fill before
# every call, decode included (FORY_TEST_WS_FILL_ALL=1): call V's setting, on the nested
# file alone. Usage: gpu_w.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06w}
mkdir -p $O
FORY_TEST_WS_FILL=0xff timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_treecol.py tests/test_gpu_v9.py \
  -m gpu -q --timeout 120 --timeout-method thread --maxfail 30 > $O/pytest_ws_ff_fresh.log 2>&1
rc=$?
echo "(a) fill per call sequence: exit $rc"; tail -35 $O/pytest_ws_ff_fresh.log
grep -q -i "illegal\|aborted\|core dumped" $O/pytest_ws_ff_fresh.log && { echo "fault: stop"; exit 1; }
[ $rc -le 1 ] || exit 1
FORY_TEST_WS_FILL=0xff FORY_TEST_WS_FILL_ALL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py \
  -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_ws_ff_all.log 2>&1
echo "(b) fill before every call: exit $?"; tail -3 $O/pytest_ws_ff_all.log
exit 0
