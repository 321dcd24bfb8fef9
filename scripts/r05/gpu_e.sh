#!/bin/bash
# Round-5 step E: the staged-copy split fix (pageable pieces over 1 MiB), the varlen
# registered-vs-pageable check at 8Mi rows, and PCIe calibration (hipHostMalloc vs
# registered heap memory; per-column copies / one copy / gather kernel, +- a concurrent D2H).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05e}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py -m gpu -q -x -k "pageable_pieces or zero_copy" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/r05/dbg_var_reg.py 8388608 mixed40 > $O/dbg_var.log 2>&1
rc=$?; head -4 $O/dbg_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 scripts/microbench/bin/h2d_ab 1048576 > $O/h2d_ab_hostmalloc.json 2>&1
rc=$?; cat $O/h2d_ab_hostmalloc.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 scripts/microbench/bin/h2d_ab 1048576 reg > $O/h2d_ab_registered.json 2>&1
rc=$?; cat $O/h2d_ab_registered.json; exit $rc
