#!/bin/bash
# Round 6, call J: the fused frame-index walk vs chunk geometry (FORY_ROWFMT_IDXFRAMES:
# frames per chunk, chunk bytes = that x the mean frame rounded to 256) -- is the walk
# bound by lanes reading 8 KiB-strided addresses?
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
export PYTHONUNBUFFERED=1
for per in 16 15 17 8 12 24 33; do
  for k in 1 0; do
    FORY_ROWFMT_IDXFRAMES=$per FORY_ROWFMT_STREAMSIZES=$k timeout -k 10 300 python -u bench.py --config mixed40 --frame \
      --no-cpu-baseline --steps 5 --warmup 2 > $O/m_${per}_k$k.json 2> $O/m_${per}_k$k.err || exit $?
    python3 -c "import json;d=json.load(open('$O/m_${per}_k$k.json'));print('per $per k$k', d['value'], d['kernels_ms']['sizes_avg'])"
  done
done
