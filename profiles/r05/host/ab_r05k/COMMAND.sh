#!/bin/bash
# Round-5 step K: host staging with non-temporal pool copies (in-tree 16 MiB x 8 vs 4 MiB x
# 16), pageable; registered A/B in-tree (registration-table mappings) vs runtime queries per copy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05k}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py -m gpu -q -x -k "pageable or registered or staged" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in intree st4x16; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    HOST_MEM=pageable timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/pg_${v}_$r.json 2> $O/pg_${v}_$r.err
    rc=$?; echo "pageable $v $r: $(python3 -c "import json; d=json.load(open('$O/pg_${v}_$r.json'))['raw']; print(d['value_GiBs'], d['encode_s'], d['decode_s'])")"; [ $rc -eq 0 ] || exit $rc
  done
  for v in intree queries; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/reg_${v}_$r.json 2> $O/reg_${v}_$r.err
    rc=$?; echo "registered $v $r: $(python3 -c "import json; d=json.load(open('$O/reg_${v}_$r.json'))['raw']; print(d['value_GiBs'], d['encode_s'], d['decode_s'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
unset FORY_ROWFMT_LIB
HOST_MEM=pageable timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_pageable.json 2> $O/host_var_pageable.err
rc=$?; echo "var pageable exit $rc"; cat $O/host_var_pageable.json; exit $rc
