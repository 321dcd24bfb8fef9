#!/bin/bash
# Round-3 closing profiles: Struct104 (C4 bench command), Mixed 16M and Nested 8M — kernel
# trace + stats, FETCH_SIZE and WRITE_SIZE passes (scripts/profile.sh), and the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 400 python bench.py > gpurun_out/final/bench_struct104_b.json 2> gpurun_out/final/bench_struct104_b.err
rc=$?; echo "bench exit $rc"; cut -c1-200 gpurun_out/final/bench_struct104_b.json; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/final/prof_struct104 bash scripts/profile.sh > gpurun_out/final/prof_struct104.log 2>&1
rc=$?; echo "prof struct104 exit $rc"; tail -3 gpurun_out/final/prof_struct104.log; [ $rc -eq 0 ] || exit $rc
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=gpurun_out/final/prof_$cfg BENCH_EXTRA="--config $cfg" ROWS=$rows bash scripts/profile.sh > gpurun_out/final/prof_$cfg.log 2>&1
  rc=$?; echo "prof $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
