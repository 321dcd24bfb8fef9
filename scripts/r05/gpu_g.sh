#!/bin/bash
# Round-5 step G: tree-engine container encode with item inputs in flight (parity + Holder /
# BeanA rates), then the fixed-width host path timelines (step F).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05g}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_treecol.py tests/test_gpu_nested.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/shapes.log 2>&1
rc=$?; grep "^{" $O/shapes.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r05/gpu_f.sh ${1:-r05g}
