#!/bin/bash
# Host path: pinned registrations verified once per call (cache), host tests + rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_windows.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
HOST_MEM=registered timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed.json 2> $O/host_fixed.err
rc=$?; cat $O/host_fixed.json; exit $rc
