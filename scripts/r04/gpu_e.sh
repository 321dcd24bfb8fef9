#!/bin/bash
# Where the varlen tile kernels' time goes (timing only, FORY_ROWFMT_DBGSKIP): loads alone,
# everything but the encode's image store, full; Mixed and Nested; round-trip check off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04e
mkdir -p $O
for cfg in mixed40 nested; do
  for sk in 0 1 2; do
    FORY_ROWFMT_DBGSKIP=$sk timeout -k 10 200 python scripts/r04/kernel_times.py $cfg > $O/skip_${cfg}_$sk.json 2> $O/skip_${cfg}_$sk.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/skip_${cfg}_$sk.err; exit $rc; }
    echo "$cfg skip=$sk $(cat $O/skip_${cfg}_$sk.json)"
  done
done
