#!/bin/bash
# Round-5 step T: Nested 8Mi encode and decode under the engine / budget knobs (no rebuild): staging
# slot bytes, register staging, waves per tile; two alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05t}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in default stg1024 stg4096 decregs nw4 cap; do
    unset FORY_ROWFMT_VARSTG FORY_ROWFMT_DECREGS FORY_ROWFMT_VARNW FORY_ROWFMT_VARFIT
    case $v in
      stg1024) export FORY_ROWFMT_VARSTG=1024;; stg4096) export FORY_ROWFMT_VARSTG=4096;;
      decregs) export FORY_ROWFMT_DECREGS=1;; nw4) export FORY_ROWFMT_VARNW=4;; cap) export FORY_ROWFMT_VARFIT=1;;
    esac
    timeout -k 10 200 python bench.py --config nested --steps 5 --warmup 2 --no-cpu-baseline > $O/n_${v}_$r.json 2> $O/n_${v}_$r.err
    rc=$?; echo "$v $r: $(python3 -c "import json; d=json.load(open('$O/n_${v}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_call_avg'], k['decode_call_avg'], k['decode_avg'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
