#!/bin/bash
# Round-5 step Z: Struct104 (64Mi windows) on the final library (e3cdc644) and the build
# before it (f83f48fa, lib_ab/f83f), alternating on one box, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05z}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in e3cd f83f; do
    if [ $v = f83f ]; then export FORY_ROWFMT_LIB=$PWD/fury_amd/lib_ab/f83f/libfory_rowfmt.so; else unset FORY_ROWFMT_LIB; fi
    timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > $O/s_${v}_$r.json 2> $O/s_${v}_$r.err
    rc=$?; echo "$v $r: $(python3 -c "import json; d=json.load(open('$O/s_${v}_$r.json')); print(d['value'], d['kernels_ms'], d['lib_sha16'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
