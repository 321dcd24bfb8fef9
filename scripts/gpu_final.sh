#!/bin/bash
# Round-end check on the committed tree: full GPU suite, smoke(), default bench,
# varlen benches, 2-rank rehearsal of bench.py --gpus 2 (gloo, both ranks on cuda:0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; echo "bench exit $rc"; cut -c1-400 gpurun_out/bench_final.json; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench_final_$cfg.json 2> gpurun_out/bench_final_$cfg.err
  rc=$?; echo "bench $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --oversubscribe --total-rows 16777216 --weak-rows 4194304 \
  --steps 3 --warmup 1 > gpurun_out/bench_final_2rank.json 2> gpurun_out/bench_final_2rank.err
rc=$?; echo "2-rank bench exit $rc"; exit $rc
