#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE passes for the varlen configs; per-launch traffic of
# their encode / decode-values kernels into gpurun_out/pmc_latest.json (merged per config key).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=gpurun_out/prof_$cfg BENCH_EXTRA="--config $cfg" ROWS=$rows bash scripts/profile.sh > gpurun_out/prof_$cfg.log 2>&1
  rc=$?; echo "prof $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_to_traffic.py gpurun_out/prof_$cfg/summary.json $cfg:$rows:0 gpurun_out/pmc_latest.json || exit 1
done
