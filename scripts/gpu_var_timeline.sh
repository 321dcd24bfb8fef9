#!/bin/bash
# Phase timelines of the cooperative varlen kernels (FORY_ROWFMT_VARPROF=1) for the
# BASELINE varlen configs; JSON to gpurun_out/timeline_<config>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CONFIGS:-nested mixed40}; do
  timeout -k 10 200 python scripts/var_timeline.py $cfg > gpurun_out/timeline_$cfg.json 2> gpurun_out/timeline_$cfg.err || { tail -5 gpurun_out/timeline_$cfg.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/timeline_$cfg.json'))
for k,v in d.items():
    print(k, 'life', v.get('tile_life_us_median'), 'resident', v.get('avg_resident_tiles'), 'span', v.get('kernel_span_us'), {a:b['median_us'] for a,b in v.items() if isinstance(b,dict)})
"
done
