#!/bin/bash
# GPU-box check: parity tests, then (only if they pass) the default bench and a
# 2-rank rehearsal of the multi-GPU bench path (gloo, both ranks on cuda:0).
# Every GPU step has its own time limit; nothing runs after a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out}
{ nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; command -v java || echo "java: absent"; } > $OUT/host_cpu.txt 2>&1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest_gpu.log
tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 8} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "bench exit $rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_RANKS" ] && exit 0
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --oversubscribe --total-rows 16777216 --weak-rows 4194304 \
  --steps 3 --warmup 1 > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err
rc=$?
echo "2-rank bench exit $rc"; cat $OUT/bench_2rank.json; tail -3 $OUT/bench_2rank.err
exit $rc
