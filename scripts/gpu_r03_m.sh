#!/bin/bash
# Round 3: full GPU suite after coalesced scans + string copy kernel, nested-shape
# throughput, varlen benches (batched tile-total scans), kernel stats of the nested shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03m_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r03m_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_nested_shapes.py 2097152 > gpurun_out/r03m_nested.log 2>&1
rc=$?; echo "nested bench exit $rc"; tail -1 gpurun_out/r03m_nested.log; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03m_$cfg.json 2> gpurun_out/r03m_$cfg.err
  rc=$?; echo "bench $cfg exit $rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['kernels_ms'])" gpurun_out/r03m_$cfg.json; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03m_prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_nested_shapes.py 524288 > $GRAFT_REPO_ROOT/gpurun_out/r03m_prof.log 2>&1
echo "rocprof exit $?"
