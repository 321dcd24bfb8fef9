#!/bin/bash
# Round 3: kernel trace of the nested-shape bench (holder, bean_a at 2M records) after the decode rework.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03q_prof -o run -- python3 $R/scripts/bench_nested_shapes.py 524288 lists,bean_a > $R/gpurun_out/r03q_prof.log 2>&1
echo "rocprof exit $?"
