#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/var_timeline.py mixed40 > gpurun_out/timeline_mixed.json 2> gpurun_out/timeline.err
rc=$?; echo "timeline exit $rc"; tail -3 gpurun_out/timeline.err; cat gpurun_out/timeline_mixed.json; exit $rc
