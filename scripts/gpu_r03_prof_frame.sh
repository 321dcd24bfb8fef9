#!/bin/bash
# Closing-build rocprof of the frame-stream benches (decode from the stream alone, frame
# index included): kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=gpurun_out/final/prof_${cfg}_frame BENCH_EXTRA="--config $cfg --frame" ROWS=$rows bash scripts/profile.sh > gpurun_out/final/prof_${cfg}_frame.log 2>&1
  rc=$?; echo "prof $cfg frame exit $rc"; [ $rc -eq 0 ] || exit $rc
done
