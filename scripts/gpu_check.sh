#!/bin/bash
# GPU-box check: parity tests, then (only if they pass) a short bench.
# Every GPU step has its own time limit; nothing runs after a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; } > gpurun_out/host_cpu.txt 2>&1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 8} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench exit $rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
