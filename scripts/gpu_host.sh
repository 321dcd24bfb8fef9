#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/host_inclusive.py 8388608 1048576 > gpurun_out/host_inclusive.json 2> gpurun_out/host_inclusive.err
rc=$?; echo "host exit $rc"; cat gpurun_out/host_inclusive.json; tail -3 gpurun_out/host_inclusive.err
[ $rc -eq 0 ] || exit $rc
# one rank through torchrun (the driver's N>1 launch form), to exercise the distributed init path
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --rows 8388608 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err
rc=$?; echo "torchrun exit $rc"; cat gpurun_out/bench_torchrun.json; tail -3 gpurun_out/bench_torchrun.err
exit $rc
