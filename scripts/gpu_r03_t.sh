#!/bin/bash
# Round 3: nullable fixed-width decode (validity from the gathers' null bits) — parity, then A/B against the base build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03t_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r03t_pytest.log; [ $rc -eq 0 ] || exit $rc
B=$GRAFT_REPO_ROOT/fury_amd/lib/libfory_rowfmt_base.so
for i in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export FORY_ROWFMT_LIB=$B; else unset FORY_ROWFMT_LIB; fi
    timeout -k 10 120 python scripts/bench_nullable_fixed.py > gpurun_out/r03t_$lib$i.json 2>&1
    rc=$?; echo "nullable $lib $i exit $rc: $(cat gpurun_out/r03t_$lib$i.json | tail -1 | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
  done
done
