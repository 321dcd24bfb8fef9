#!/bin/bash
# Round 3: columnar engine after the decode level rework + inline flat beans: parity, nested-shape throughput, kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_treecol.py tests/test_gpu_nested.py tests/test_gpu_host.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03f_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/r03f_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_nested_shapes.py 2097152 > gpurun_out/r03f_nested.log 2>&1
rc=$?; echo "nested bench exit $rc"; tail -1 gpurun_out/r03f_nested.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03f_prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_nested_shapes.py 524288 > $GRAFT_REPO_ROOT/gpurun_out/r03f_prof.log 2>&1
echo "rocprof exit $?"
