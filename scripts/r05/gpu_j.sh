#!/bin/bash
# Round-5 step J: pageable staging geometry A/B (block MiB x blocks; in-tree = 16 x 8), then
# FETCH / WRITE passes of the tree engine on BeanA (per-kernel HBM bytes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05j}
R=$PWD
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in intree st4x16 st8x16 st4x8; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    HOST_MEM=pageable timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/pg_${v}_$r.json 2> $O/pg_${v}_$r.err
    rc=$?; echo "$v $r: $(python3 -c "import json; d=json.load(open('$O/pg_${v}_$r.json'))['raw']; print(d['value_GiBs'], d['encode_s'], d['decode_s'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
unset FORY_ROWFMT_LIB
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/tree_$c -o p -- python3 $R/scripts/bench_nested_shapes.py 2097152 bean_a,holder > $O/tree_$c.log 2>&1
  rc=$?; echo "pmc $c exit $rc"; [ $rc -eq 0 ] || exit $rc
done
