#!/bin/bash
# Round 6, call K: frames per frame-index chunk, 16 (default) vs 20 / 24, Mixed and Nested
# frame streams, three alternating rounds (FORY_ROWFMT_IDXFRAMES).
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
bash scripts/r06/gpu_box.sh || exit $?
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for cfg in mixed40 nested; do
    for per in 16 20 24; do
      FORY_ROWFMT_IDXFRAMES=$per timeout -k 10 300 python -u bench.py --config $cfg --frame --no-cpu-baseline \
        > $O/${cfg}_${per}_$r.json 2> $O/${cfg}_${per}_$r.err || exit $?
      python3 -c "import json;d=json.load(open('$O/${cfg}_${per}_$r.json'));k=d['kernels_ms'];print('$cfg per $per r$r', d['value'], k['frame_index_avg'], k['decode_avg'])"
    done
  done
done
