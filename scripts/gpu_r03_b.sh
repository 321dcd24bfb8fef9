#!/bin/bash
# Round 3, call B: full GPU suite (encode v6 default for flat plans), then Mixed / Nested
# benches with v6 on and off (same process build, plan-time knob), then the counter
# profile of the varlen benches. Every GPU step has its own limit; stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/r03b_pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in mixed40 nested; do
  for e6 in 1 0; do
    FORY_ROWFMT_ENC6=$e6 FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03b_$cfg.e6_$e6.json 2> gpurun_out/r03b_$cfg.e6_$e6.err
    rc=$?; echo "bench $cfg enc6=$e6 exit $rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['kernels_ms'])" gpurun_out/r03b_$cfg.e6_$e6.json; [ $rc -eq 0 ] || exit $rc
  done
done
for wg in 0 512; do
  FORY_ROWFMT_NULWG=$wg timeout -k 10 120 python scripts/bench_nullable_fixed.py > gpurun_out/r03_nul_$wg.json 2>&1
  rc=$?; echo "nullable wg=$wg exit $rc"; cat gpurun_out/r03_nul_$wg.json; [ $rc -eq 0 ] || exit $rc
done
SQ=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE
for spec in mixed40:16777216 nested:8388608; do
  cfg=${spec%%:*}; rows=${spec##*:}
  OUT=gpurun_out/r03_prof_$cfg BENCH_EXTRA="--config $cfg" ROWS=$rows EXTRA_PMC=$SQ bash scripts/profile.sh > gpurun_out/r03_prof_$cfg.log 2>&1
  rc=$?; echo "prof $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
