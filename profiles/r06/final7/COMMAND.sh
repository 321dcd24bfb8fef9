#!/bin/bash
# Round 6, call U: the whole GPU suite in the order that failed in r06final5 (host-path files
# after every device test, FORY_TEST_HOST_LAST=1), on the library with the arena memset fix,
# then smoke. Usage: gpu_u.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06final7}
mkdir -p $O
FORY_TEST_HOST_LAST=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
sha256sum fury_amd/lib/libfory_rowfmt.so | cut -c1-16 > $O/lib_sha16.txt
