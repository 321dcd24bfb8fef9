#!/bin/bash
# Round 3, call A: decimal + host tests on the GPU, then a counter profile of the varlen
# benches (Mixed 16M, Nested 8M): kernel trace (resources), FETCH/WRITE, and one SQ pass
# of wave-time buckets and LDS bank conflicts. Every GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r03a_pytest.log; [ $rc -eq 0 ] || exit $rc
SQ=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=gpurun_out/r03_prof_$cfg BENCH_EXTRA="--config $cfg" ROWS=$rows EXTRA_PMC=$SQ bash scripts/profile.sh > gpurun_out/r03_prof_$cfg.log 2>&1
  rc=$?; echo "prof $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
# nullable fixed-width: default vs 512-thread workgroups (FORY_ROWFMT_NULWG, plan-time knob)
for wg in 0 512; do
  FORY_ROWFMT_NULWG=$wg timeout -k 10 120 python scripts/bench_nullable_fixed.py > gpurun_out/r03_nul_$wg.json 2>&1
  rc=$?; echo "nullable wg=$wg exit $rc"; cat gpurun_out/r03_nul_$wg.json; [ $rc -eq 0 ] || exit $rc
done
