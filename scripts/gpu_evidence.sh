#!/bin/bash
# Round evidence: parity tests, benches (raw + frame), rocprofv3 kernel trace + PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_final bash scripts/profile.sh > gpurun_out/profile.log 2>&1
rc=$?; echo "profile exit $rc"; tail -3 gpurun_out/profile.log; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_to_traffic.py gpurun_out/prof_final/summary.json struct104:67108864:0 gpurun_out/pmc_latest.json
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --frame --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_frame.json 2> gpurun_out/bench_frame.err
rc=$?; echo "bench frame exit $rc"; cat gpurun_out/bench_frame.json
[ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "bench $cfg exit $rc"; cat gpurun_out/bench_$cfg.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 0 > gpurun_out/bench_nullable.json
rc=$?; echo "bench nullable exit $rc"; cat gpurun_out/bench_nullable.json; [ $rc -eq 0 ] || exit $rc
