#!/bin/bash
# Round-3 closing run on the committed tree: full GPU suite, smoke(), default bench (C4),
# varlen benches raw + frame, the nested-shape bench, 2-rank gloo rehearsal of --gpus 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
O=gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_struct104.json 2> $O/bench_struct104.err
rc=$?; echo "bench exit $rc"; cut -c1-300 $O/bench_struct104.json; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  for fr in "" "--frame"; do
    tag=$cfg${fr:+_frame}
    timeout -k 10 300 python bench.py --config $cfg $fr --steps 10 --warmup 3 --cpu-seconds 8 > $O/bench_$tag.json 2> $O/bench_$tag.err
    rc=$?; echo "bench $tag exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -u scripts/bench_nested_shapes.py 2097152 > $O/nested_shapes_2M.log 2>&1
rc=$?; echo "nested shapes exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --oversubscribe --total-rows 16777216 --weak-rows 4194304 \
  --steps 3 --warmup 1 > $O/bench_2rank.json 2> $O/bench_2rank.err
rc=$?; echo "2-rank bench exit $rc"; exit $rc
