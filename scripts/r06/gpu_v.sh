#!/bin/bash
# Round 6, call V: do the varlen / tree-engine kernels read workspace words they did not
# write? The RowEncoder workspace is filled with 0xff before every call
# (FORY_TEST_WS_FILL, fury_amd/format/encoder.py); parity against the oracle must hold.
# 0xff makes any such int64 word -1 (an address just below its base, not a wild one).
# Usage: gpu_v.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06v}
mkdir -p $O
FORY_TEST_WS_FILL=0xff timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_treecol.py tests/test_gpu_v9.py \
  -m gpu -q --timeout 120 --timeout-method thread --maxfail 20 > $O/pytest_ws_ff.log 2>&1
rc=$?
tail -25 $O/pytest_ws_ff.log
exit $rc
