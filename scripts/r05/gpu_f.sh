#!/bin/bash
# Round-5 step F: timelines of the fixed-width host path (kernel + memory-copy trace),
# per-slice copies (HOSTPATH=2) and gather launches (HOSTPATH=0), registered buffers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05f}
mkdir -p $O
R=$PWD
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
for hp in 2 0; do
  FORY_ROWFMT_HOSTPATH=$hp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $O/trace_hp$hp -o t -- python3 $R/scripts/host_native.py 4194304 1048576 > $O/trace_hp$hp.log 2>&1
  rc=$?; echo "hostpath $hp exit $rc"; grep round_trip $O/trace_hp$hp.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
