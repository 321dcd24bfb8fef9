#!/bin/bash
# Round 3: HBM traffic of the columnar encode (holder, bean_a at 524288 rows), one PMC pass each.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/r03d_fetch -o run -- python3 $R/scripts/bench_nested_shapes.py 524288 holder,bean_a --encode-only > $R/gpurun_out/r03d_fetch.log 2>&1
echo "fetch exit $?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/r03d_write -o run -- python3 $R/scripts/bench_nested_shapes.py 524288 holder,bean_a --encode-only > $R/gpurun_out/r03d_write.log 2>&1
echo "write exit $?"
