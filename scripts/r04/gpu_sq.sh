#!/bin/bash
# Wave-time buckets (SQ counters, one pass of their own) of the Mixed and Nested benches on
# the closing build: encode v9 / round-3 kernel and the decode passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04sq
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=$O/prof_$cfg BENCH_EXTRA="--config $cfg" ROWS=$rows EXTRA_PMC="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS" bash scripts/profile.sh > $O/prof_$cfg.log 2>&1
  rc=$?; echo "prof $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
