#!/bin/bash
# Round-4 first GPU pass: the new memo / short-length tests, full GPU suite, smoke, default
# bench (C4 + the C2/C3 extra lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_treecol.py -x -v --timeout 120 --timeout-method thread > $O/pytest_treecol.log 2>&1
rc=$?; tail -3 $O/pytest_treecol.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; cut -c1-400 $O/bench.json; exit $rc
