#!/bin/bash
# A/B of builds of libfory_rowfmt.so on one box: bench.py per config, alternating the
# in-tree build ("new") and each LIBS entry (name:path, via FORY_ROWFMT_LIB), ROUNDS times.
# Usage: LIBS="base:fury_amd/lib_ab/libfory_rowfmt_base.so" CONFIGS="mixed40 nested" bash scripts/ab_builds.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-base:fury_amd/lib_ab/libfory_rowfmt_base.so}
for r in $(seq ${ROUNDS:-2}); do
  for cfg in ${CONFIGS:-mixed40 nested}; do
    for entry in new $LIBS; do
      name=${entry%%:*}
      if [ "$name" = new ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=${entry#*:}; fi
      timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$name.json 2>/dev/null || exit 1
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$name.json')); k=d['kernels_ms']; print('$cfg $name', d['value'], k['encode_call_avg'], k['decode_call_avg'], k['encode_avg'], k['decode_avg'])"
    done
  done
done
