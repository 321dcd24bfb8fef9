#!/bin/bash
# Round 6, call L: the host copy machinery after the drain-on-every-return change: the
# copies-only GPU test, the host and window test files, then the pageable host rates.
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_copies.py tests/test_gpu_host.py tests/test_gpu_windows.py > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_pageable.json || exit $?
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native_var.py > $O/host_var_pageable.json || exit $?
cat $O/host_*.json | cut -c1-600
