#!/bin/bash
# RCCL rehearsal on a 1-GPU box: bench.py --gpus 1 --init-dist starts one torchrun rank that
# initialises the nccl (RCCL) process group and runs the line's collectives on the device
# (init all_reduce, device all_gather_object, barriers, MAX over ranks); Struct104 16Mi rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rccl1
timeout -k 10 300 python bench.py --gpus 1 --init-dist --backend nccl --total-rows 16777216 --weak-rows 0 \
  --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rccl1/bench_rccl1.json 2> gpurun_out/rccl1/bench_rccl1.err
rc=$?; echo "rccl 1-rank bench exit $rc"; cut -c1-400 gpurun_out/rccl1/bench_rccl1.json; tail -3 gpurun_out/rccl1/bench_rccl1.err
[ $rc -eq 0 ] || exit $rc
# stdout must be the JSON line alone (RCCL's banner goes to stderr)
n=$(wc -l < gpurun_out/rccl1/bench_rccl1.json); echo "stdout lines: $n"; [ "$n" -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --oversubscribe --total-rows 16777216 --weak-rows 0 \
  --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rccl1/bench_2rank_gloo.json 2> gpurun_out/rccl1/bench_2rank_gloo.err
rc=$?; echo "gloo 2-rank bench exit $rc"; [ $rc -eq 0 ] || exit $rc
n=$(wc -l < gpurun_out/rccl1/bench_2rank_gloo.json); echo "stdout lines: $n"; [ "$n" -eq 1 ] || exit 1
