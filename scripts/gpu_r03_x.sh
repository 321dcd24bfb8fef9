#!/bin/bash
# Round 3: tree-engine tests (long strings: both copy paths) + kernel trace of bean_a at 512K.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_treecol.py -x -q -k "resume or long" --timeout 120 --timeout-method thread > gpurun_out/r03x_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r03x_pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03x_prof -o run -- python3 $R/scripts/bench_nested_shapes.py 524288 bean_a,holder > $R/gpurun_out/r03x_prof.log 2>&1
echo "rocprof exit $?"
