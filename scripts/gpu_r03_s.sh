#!/bin/bash
# Round 3: spill-image size A/B for the varlen tile kernels (plan-time knob FORY_ROWFMT_SPILLCAP).
set -o pipefail
mkdir -p gpurun_out
for spec in "nested 0" "nested 16384" "nested 24576" "mixed40 0" "mixed40 49152" "mixed40 65536"; do
  set -- $spec
  FORY_ROWFMT_SPILLCAP=$2 timeout -k 10 200 python bench.py --config $1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03s_$1_$2.json 2> gpurun_out/r03s_$1_$2.err
  rc=$?; echo "bench $1 spill=$2 exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['kernels_ms'])" gpurun_out/r03s_$1_$2.json
done
