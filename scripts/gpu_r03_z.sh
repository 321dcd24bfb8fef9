#!/bin/bash
# Round 3: encode tile image grown before the staging — varlen parity, then A/B (alternating) against the frozen build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03z_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r03z_pytest.log; [ $rc -eq 0 ] || exit $rc
B=$GRAFT_REPO_ROOT/fury_amd/lib/libfory_rowfmt_base.so
for i in 1 2; do
  for cfg in nested mixed40; do
    for lib in new base; do
      if [ $lib = base ]; then export FORY_ROWFMT_LIB=$B; else unset FORY_ROWFMT_LIB; fi
      FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03z_${cfg}_$lib$i.json 2> gpurun_out/r03z_${cfg}_$lib$i.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg $lib exit $rc"; exit $rc; }
      echo "$cfg $lib $i: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['kernels_ms']['encode_call_avg'], d['kernels_ms']['decode_call_avg'])" gpurun_out/r03z_${cfg}_$lib$i.json) $(grep 'encode' gpurun_out/r03z_${cfg}_$lib$i.err | head -1 | cut -c1-120)"
    done
  done
done
