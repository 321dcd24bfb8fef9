#!/bin/bash
# Round 6, call T: which stream torch's "stream 0" is (scripts/microbench/null_stream_probe.py),
# then the second half of the closing profiles (Nested, Nested frames) and the default bench
# line. Usage: gpu_t.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-close6}
mkdir -p $O
timeout -k 10 180 python -u scripts/microbench/null_stream_probe.py > $O/null_stream_probe.json 2>&1 || { cat $O/null_stream_probe.json; exit 1; }
cat $O/null_stream_probe.json
SPECS="nested:8388608: nested:8388608:--frame" bash scripts/r06/gpu_close.sh ${1:-close6}
