#!/bin/bash
# Round 3: columnar decode with list items batched 4 per lane in the encode: parity, nested-shape throughput.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_treecol.py tests/test_gpu_nested.py tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03y_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r03y_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_nested_shapes.py 2097152 > gpurun_out/r03y_nested.log 2>&1
rc=$?; echo "nested bench exit $rc"; tail -1 gpurun_out/r03y_nested.log
