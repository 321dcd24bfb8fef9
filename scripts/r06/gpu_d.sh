#!/bin/bash
# Round 6, call D: host path with call-scoped registration of pageable caller buffers
#  + verify mode: host tests, then host-inclusive rates.
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host.py tests/test_gpu_windows.py > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_pageable.json || exit $?
timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_registered.json || exit $?
cat $O/host_fixed_pageable.json $O/host_fixed_registered.json
