#!/bin/bash
# Round 6, call F: host path (call-scoped registration, helper thread with first-use order):
# host tests, then host-inclusive rates, pageable and registered, fixed and varlen.
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host.py tests/test_gpu_windows.py > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_pageable.json || exit $?
timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_registered.json || exit $?
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native_var.py > $O/host_var_pageable.json || exit $?
timeout -k 10 300 python -u scripts/host_native_var.py > $O/host_var_registered.json || exit $?
cat $O/host_*.json
