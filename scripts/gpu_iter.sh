#!/bin/bash
# Iteration run: GPU parity tests, microbench, in-process A/B of kernel variants, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$MICRO" ]; then
  timeout -k 10 300 ./scripts/microbench/colread > gpurun_out/colread.jsonl 2> gpurun_out/colread.err
  rc=$?; echo "colread exit $rc"; cat gpurun_out/colread.jsonl; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python scripts/ab_fixed.py 67108864 2 > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab exit $rc"; python -c "import json;d=json.load(open('gpurun_out/ab.json'));[print(k,v.get('enc_ms'),v.get('dec_ms'),v.get('enc_GBs',v.get('enc_GBs_algo')),v.get('dec_GBs')) for k,v in d.items()]"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; tail -2 gpurun_out/bench.err
exit $rc
