#!/bin/bash
# Phase timelines of encode v7 vs the round-3 encode tile kernel (FORY_ROWFMT_VARENC=1),
# Mixed and Nested, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04c
mkdir -p $O
for enc in 0 1; do
  for cfg in mixed40 nested; do
    FORY_ROWFMT_VARENC=$enc timeout -k 10 200 python scripts/var_timeline.py $cfg > $O/timeline_${cfg}_enc$enc.json 2> $O/timeline_${cfg}_enc$enc.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/timeline_${cfg}_enc$enc.err; exit $rc; }
    python3 -c "
import json; d=json.load(open('$O/timeline_${cfg}_enc$enc.json'))
for k,v in d.items():
    print('enc$enc', k, 'life', v.get('tile_life_us_median'), 'resident', v.get('avg_resident_tiles'), 'span', v.get('kernel_span_us'), {a:b['median_us'] for a,b in v.items() if isinstance(b,dict)})
"
  done
done
