#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on the closing build (gloo, both ranks on
# cuda:0), and the torchrun form of the N=1 line with the nccl (RCCL) branch initialised.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04ranks
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --oversubscribe --total-rows 16777216 --weak-rows 4194304 \
  --steps 3 --warmup 1 > $O/bench_2rank.json 2> $O/bench_2rank.err
rc=$?; echo "2-rank exit $rc"; cut -c1-300 $O/bench_2rank.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --init-dist --steps 3 --warmup 1 > $O/bench_rccl1.json 2> $O/bench_rccl1.err
rc=$?; echo "rccl1 exit $rc"; cut -c1-300 $O/bench_rccl1.json; exit $rc
