#!/bin/bash
# Round 6, call A: the pinned-block coherence probe and the
# debug-bounds library over the host + parity test files (item 2).
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 scripts/microbench/bin/pinned_probe 8 > $O/probe_default.jsonl || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 400 scripts/microbench/bin/pinned_probe 8 > $O/probe_nosdma.jsonl || exit $?
FORY_ROWFMT_LIB=$PWD/fury_amd/lib/debug/libfory_rowfmt.so timeout -k 10 900 python -u -m pytest -x -q \
  --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host.py tests/test_gpu_parity.py \
  > $O/pytest_debug_bounds.log 2>&1 || exit $?
echo done
