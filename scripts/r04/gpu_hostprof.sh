#!/bin/bash
# Host fixed-width path: kernel + memory-copy trace of scripts/host_native.py (registered
# buffers), to see where the call's time goes (copies, kernels, gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04hostprof
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o host --output-format csv -- python3 scripts/host_native.py 8388608 1048576 > $O/host_fixed.json 2> $O/host_fixed.err
rc=$?; echo "exit $rc"; cat $O/host_fixed.json; ls -R $O/trace | head -20; exit $rc
