#!/bin/bash
# Full GPU suite in ONE process (test_gpu_host's registration cases included) + smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05a}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; exit $rc
