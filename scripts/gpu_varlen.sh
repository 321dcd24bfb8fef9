#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in mixed40 nested; do
  timeout -k 10 500 python bench.py --config $cfg --steps 5 --warmup 2 --cpu-seconds 6 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "$cfg exit $rc"; cat gpurun_out/bench_$cfg.json; tail -3 gpurun_out/bench_$cfg.err; [ $rc -eq 0 ] || exit $rc
done
OUT=gpurun_out/prof_mixed BENCH_EXTRA="--config mixed40" ROWS=16777216 bash scripts/profile.sh > gpurun_out/prof_mixed.log 2>&1
echo "prof mixed exit $?"
