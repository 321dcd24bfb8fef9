#!/bin/bash
# A/B of the encode staging size (adaptive vs FORY_ROWFMT_VARSTG) on the varlen configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in nested mixed40 mixed40_long; do
  for stg in adaptive 2048 4096; do
    if [ $stg = adaptive ]; then unset FORY_ROWFMT_VARSTG; else export FORY_ROWFMT_VARSTG=$stg; fi
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$c_$stg.json 2> gpurun_out/ab.err || exit 1
    echo "$c stg=$stg $(grep -o 'kernels_ms[^}]*' gpurun_out/ab_$c_$stg.json)"
  done
done
