#!/bin/bash
# Round 3: Nested tile-image size A/B (plan-time knob FORY_ROWFMT_VARCAP; 0 = fitted to the mean row).
set -o pipefail
mkdir -p gpurun_out
for cap in 0 10752 11776 12800; do
  FORY_ROWFMT_VARCAP=$cap FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config nested --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03u_$cap.json 2> gpurun_out/r03u_$cap.err
  rc=$?; echo "bench nested cap=$cap exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['kernels_ms'])" gpurun_out/r03u_$cap.json
  grep "tile kernel" gpurun_out/r03u_$cap.err | sort | uniq -c | head -4
done
