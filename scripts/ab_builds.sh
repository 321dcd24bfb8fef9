#!/bin/bash
# A/B of two builds of libfory_rowfmt.so on one box: bench.py per config, alternating
# base (FORY_ROWFMT_LIB=$BASE) and the in-tree build, ROUNDS times.
# Usage: BASE=fury_amd/lib_ab/libfory_rowfmt_base.so CONFIGS="mixed40 nested" bash scripts/ab_builds.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BASE=${BASE:-fury_amd/lib_ab/libfory_rowfmt_base.so}
for r in $(seq ${ROUNDS:-2}); do
  for cfg in ${CONFIGS:-mixed40 nested}; do
    for which in base new; do
      if [ $which = base ]; then export FORY_ROWFMT_LIB=$BASE; else unset FORY_ROWFMT_LIB; fi
      timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$which.json 2>/dev/null || exit 1
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$which.json')); k=d['kernels_ms']; print('$cfg $which', d['value'], k['encode_call_avg'], k['decode_call_avg'], k['encode_avg'], k['decode_avg'])"
    done
  done
done
