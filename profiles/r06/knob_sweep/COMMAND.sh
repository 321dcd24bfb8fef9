#!/bin/bash
# Round 6, call P: existing launch knobs against the defaults on Nested and Mixed (raw), two
# alternating rounds: waves per tile (VARNW) and XCD tile runs (VARXCD).
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for cfg in nested mixed40; do
    for knobs in "X=0" "FORY_ROWFMT_VARNW=4" "FORY_ROWFMT_VARNW=2" "FORY_ROWFMT_VARXCD=-1" "FORY_ROWFMT_VARXCD=8"; do
      tag=$(echo "$knobs" | tr '=' '_')
      env $knobs timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline > $O/${cfg}_${tag}_$r.json 2>/dev/null || exit $?
      python3 -c "import json;d=json.load(open('$O/${cfg}_${tag}_$r.json'));k=d['kernels_ms'];print('$cfg $knobs r$r', d['value'], k['encode_call_avg'], k['decode_call_avg'])"
    done
  done
done
